// Tuning build of csrc/qstep_ws.hip: the next tile's windows issued after Q(x)'s layer 2 (WS_PF_POS 1).
// st_qstep_ws_launch_pf1 (engine.step_variant = "pf1" with step_kernel "ws").
#define WS_PF_POS 1
#define WS_NS ws_pf1
#define WS_API(name) name##_pf1
#include "qstep_ws.hip"
