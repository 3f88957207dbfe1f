// A/B build of csrc/qstep_ws.hip (correct results), round 6: #define WS_PAR 1 
// st_qstep_ws_launch_par (engine.step_variant = "par").
#define WS_PAR 1
#define WS_NS ws_par
#define WS_API(name) name##_par
#include "../qstep_ws.hip"
