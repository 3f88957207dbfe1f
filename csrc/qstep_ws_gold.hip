// Tuning build of csrc/qstep_ws.hip: the gradient waves' v4 fragment order (each phase reads what it
// needs when it starts).  st_qstep_ws_launch_gold (engine.step_variant = "gold" with step_kernel "ws").
#define WS_GPIPE 0
#define WS_GPAIR 0
#define WS_NS ws_gold
#define WS_API(name) name##_gold
#include "qstep_ws.hip"
