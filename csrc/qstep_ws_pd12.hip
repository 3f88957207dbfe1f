// Tuning / timing build of csrc/qstep_ws.hip (WS_PD1 12).
// st_qstep_ws_launch_pd12 (engine.step_variant = "pd12" with step_kernel "ws").
#define WS_PD1 12
#define WS_NS ws_pd12
#define WS_API(name) name##_pd12
#include "qstep_ws.hip"
