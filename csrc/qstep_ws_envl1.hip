// Tuning build of csrc/qstep_ws.hip: the env-state prefetch (tile k + 2) issued at layer 1's start.
// st_qstep_ws_launch_envl1 (engine.step_variant = "envl1" with step_kernel "ws").
#define WS_ENV_AT_L1 1
#define WS_NS ws_envl1
#define WS_API(name) name##_envl1
#include "qstep_ws.hip"
