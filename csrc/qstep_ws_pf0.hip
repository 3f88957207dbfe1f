// Tuning build of csrc/qstep_ws.hip: the next tile's price windows issued at Q(x')'s layer 2 (WS_PF_POS 0).
// st_qstep_ws_launch_pf0 (engine.step_variant = "pf0" with step_kernel "ws").
#define WS_PF_POS 0
#define WS_NS ws_pf0
#define WS_API(name) name##_pf0
#include "qstep_ws.hip"
