// A/B build of csrc/qstep_ws.hip: ring-wait poll loops unrolled by 2.
#define WS_WAIT_UNROLL 2
#define WS_NS ws_wunroll2
#define WS_API(name) name##_wunroll2
#include "../qstep_ws.hip"
