// Tuning build of csrc/qstep_ws.hip: the env-state prefetch (tile k + 2) issued after the slot claim.
// st_qstep_ws_launch_envslot (engine.step_variant = "envslot" with step_kernel "ws").
#define WS_ENV_AT_L1 0
#define WS_NS ws_envslot
#define WS_API(name) name##_envslot
#include "qstep_ws.hip"
