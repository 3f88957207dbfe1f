// Tuning build of csrc/qstep_ws.hip: gradient waves read X fragments 1 dW0 step ahead (production: 3).
// st_qstep_ws_launch_gx1 (engine.step_variant = "gx1" with step_kernel "ws").
#define WS_GX 1
#define WS_NS ws_gx1
#define WS_API(name) name##_gx1
#include "qstep_ws.hip"
