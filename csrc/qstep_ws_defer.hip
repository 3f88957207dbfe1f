// Tuning build of csrc/qstep_ws.hip: windows issued after Q(x)'s layer 2 and the env-state write-back
// deferred past the next tile's window wait (measured 2.6 % slower than the production schedule on one
// box, profiles/r3_ws_ab.md).  st_qstep_ws_launch_defer (engine.step_variant = "defer", step_kernel "ws").
#define WS_PF_POS 1
#define WS_WB_DEFER 1
#define WS_NS ws_defer
#define WS_API(name) name##_defer
#include "qstep_ws.hip"
