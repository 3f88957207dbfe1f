// Debug build of csrc/qstep_ws.hip: data-wave stamps with the gradient waves skipping their work (wrong
// results) -- the data wave's phases without any gradient-wave interference.
// st_qstep_ws_launch_gskipst (engine.step_variant = "gskipst" with step_kernel "ws").
#define WS_STAMPS 1
#define WS_GSKIP 1
#define WS_PD1 6
#define WS_NS ws_gskipst
#define WS_API(name) name##_gskipst
#include "../qstep_ws.hip"
