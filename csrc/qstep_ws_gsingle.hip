// Tuning build of csrc/qstep_ws.hip: gradient waves take one ring slot at a time (K = 16 MFMAs).
// st_qstep_ws_launch_gsingle (engine.step_variant = "gsingle" with step_kernel "ws").
#define WS_GPAIR 0
#define WS_NS ws_gsingle
#define WS_API(name) name##_gsingle
#include "qstep_ws.hip"
