// Tuning build of csrc/qstep_ws.hip: dZ2's LDS fragments read after TD (WS_DZ_EARLY 0).
// st_qstep_ws_launch_dzlate (engine.step_variant = "dzlate" with step_kernel "ws").
#define WS_DZ_EARLY 0
#define WS_NS ws_dzlate
#define WS_API(name) name##_dzlate
#include "qstep_ws.hip"
