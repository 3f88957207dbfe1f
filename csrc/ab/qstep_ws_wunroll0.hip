// A/B build of csrc/qstep_ws.hip: ring-wait poll loops not unrolled (the first round-4 form, 0.8-0.9 % slower).
#define WS_WAIT_UNROLL 0
#define WS_NS ws_wunroll0
#define WS_API(name) name##_wunroll0
#include "../qstep_ws.hip"
