// Tuning / timing build of csrc/qstep_ws.hip (WS_NOPHIL 1).
// st_qstep_ws_launch_nophil (engine.step_variant = "nophil" with step_kernel "ws").
#define WS_NOPHIL 1
#define WS_NS ws_nophil
#define WS_API(name) name##_nophil
#include "../qstep_ws.hip"
