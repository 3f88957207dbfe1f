// Tuning build of csrc/qstep_ws.hip: the env-state write-back issued at TD, after the next tile's window
// loads (the production position before round 3's A/B; WS_WBE 0).
// st_qstep_ws_launch_wbtd (engine.step_variant = "wbtd" with step_kernel "ws").
#define WS_WBE 0
#define WS_NS ws_wbtd
#define WS_API(name) name##_wbtd
#include "qstep_ws.hip"
