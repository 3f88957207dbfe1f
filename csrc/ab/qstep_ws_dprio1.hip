// A/B build of csrc/qstep_ws.hip (correct results), round 6: #define WS_DPRIO 1 
// st_qstep_ws_launch_dprio1 (engine.step_variant = "dprio1").
#define WS_DPRIO 1
#define WS_NS ws_dprio1
#define WS_API(name) name##_dprio1
#include "../qstep_ws.hip"
