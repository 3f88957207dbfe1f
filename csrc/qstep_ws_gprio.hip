// Tuning build of csrc/qstep_ws.hip (WS_GPRIO 2: wave issue priority).
// st_qstep_ws_launch_gprio (engine.step_variant = "gprio" with step_kernel "ws").
#define WS_GPRIO 2
#define WS_NS ws_gprio
#define WS_API(name) name##_gprio
#include "qstep_ws.hip"
