// Timing build of csrc/qstep_ws.hip (wrong results; never used for training): layer 1
// run twice per tile -- the time over the production build is that phase's cost in context.
// st_qstep_ws_launch_l1x2 (engine.step_variant = "l1x2" with step_kernel "ws").
#define WS_L1REP 2
#define WS_NS ws_l1x2
#define WS_API(name) name##_l1x2
#include "../qstep_ws.hip"
