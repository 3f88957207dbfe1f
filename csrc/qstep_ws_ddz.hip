// Tuning build of csrc/qstep_ws.hip: the data waves form dZ2 and publish it in the slot (WS_GDZ 0).
// st_qstep_ws_launch_ddz (engine.step_variant = "ddz" with step_kernel "ws").
#define WS_GDZ 0
#define WS_NS ws_ddz
#define WS_API(name) name##_ddz
#include "qstep_ws.hip"
