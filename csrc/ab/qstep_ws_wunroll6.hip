// A/B build of csrc/qstep_ws.hip: ring-wait poll loops unrolled by 6 (the round-3 kernel's inline loops were unrolled 6x).
#define WS_WAIT_UNROLL 6
#define WS_NS ws_wunroll6
#define WS_API(name) name##_wunroll6
#include "../qstep_ws.hip"
