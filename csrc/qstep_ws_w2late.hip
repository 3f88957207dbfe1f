// Tuning build of csrc/qstep_ws.hip: the output layers' W2 fragments read at the output (WS_W2_EARLY 0).
// st_qstep_ws_launch_w2late (engine.step_variant = "w2late" with step_kernel "ws").
#define WS_W2_EARLY 0
#define WS_NS ws_w2late
#define WS_API(name) name##_w2late
#include "qstep_ws.hip"
