// Tuning build of csrc/qstep_ws.hip (WS_DPRIO 2: wave issue priority).
// st_qstep_ws_launch_dprio (engine.step_variant = "dprio" with step_kernel "ws").
#define WS_DPRIO 2
#define WS_NS ws_dprio
#define WS_API(name) name##_dprio
#include "qstep_ws.hip"
