// A/B build of csrc/qstep_ws.hip (correct results), round 6: #define WS_PAR 1 #define WS_DPRIO 1 
// st_qstep_ws_launch_pardprio (engine.step_variant = "pardprio").
#define WS_PAR 1
#define WS_DPRIO 1
#define WS_NS ws_pardprio
#define WS_API(name) name##_pardprio
#include "../qstep_ws.hip"
