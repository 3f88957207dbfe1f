// Tuning build of csrc/qstep_ws.hip: window features as a multiply then a subtract (two roundings, the
// production form before round 3's fma A/B; WS_FMA_FEAT 0).
// st_qstep_ws_launch_fsub (engine.step_variant = "fsub" with step_kernel "ws").
#define WS_FMA_FEAT 0
#define WS_NS ws_fsub
#define WS_API(name) name##_fsub
#include "qstep_ws.hip"
