// Tuning / timing build of csrc/qstep_ws.hip: no env-state write-back (wrong results).
// st_qstep_ws_launch_nowb (engine.step_variant = "nowb" with step_kernel "ws").
#define WS_NOWB 1
#define WS_NS ws_nowb
#define WS_API(name) name##_nowb
#include "../qstep_ws.hip"
