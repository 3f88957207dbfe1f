// Tuning build of csrc/qstep_ws.hip: windows issued at Q(x')'s layer 2 and the env-state stores issued at
// TD (no deferral) -- the schedule before the deferred write-back, kept for A/B on one box.
// st_qstep_ws_launch_old (engine.step_variant = "old" with step_kernel "ws").
#define WS_PF_POS 0
#define WS_WB_DEFER 0
#define WS_NS ws_old
#define WS_API(name) name##_old
#include "qstep_ws.hip"
