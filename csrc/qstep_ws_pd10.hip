// Tuning build of csrc/qstep_ws.hip: layer-1 W0 fragment pairs 10 ahead (WS_PD1 10, production before the r4y A/B).
// st_qstep_ws_launch_pd10 (engine.step_variant = "pd10" with step_kernel "ws").
#define WS_PD1 10
#define WS_NS ws_pd10
#define WS_API(name) name##_pd10
#include "qstep_ws.hip"
