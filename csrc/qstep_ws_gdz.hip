// Tuning build of csrc/qstep_ws.hip: the gradient waves form dZ2 (WS_GDZ 1) -- measured 13 % slower.
// st_qstep_ws_launch_gdz (engine.step_variant = "gdz" with step_kernel "ws").
#define WS_GDZ 1
#define WS_NS ws_gdz
#define WS_API(name) name##_gdz
#include "qstep_ws.hip"
