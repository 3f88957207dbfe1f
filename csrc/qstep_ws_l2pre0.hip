// Tuning build of csrc/qstep_ws.hip: no layer-2 W1 fragment pre-read (WS_L2PRE 0, production before round 3's A/B).
// st_qstep_ws_launch_l2pre0 (engine.step_variant = "l2pre0" with step_kernel "ws").
#define WS_L2PRE 0
#define WS_NS ws_l2pre0
#define WS_API(name) name##_l2pre0
#include "qstep_ws.hip"
