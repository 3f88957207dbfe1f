// Tuning build of csrc/qstep_ws.hip: 6 layer-2 W1 fragments pre-read before the slot claim (WS_L2PRE 6).
// st_qstep_ws_launch_l2pre6 (engine.step_variant = "l2pre6" with step_kernel "ws").
#define WS_L2PRE 6
#define WS_NS ws_l2pre6
#define WS_API(name) name##_l2pre6
#include "qstep_ws.hip"
