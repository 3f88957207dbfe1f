// A/B build of csrc/qstep_ws.hip: price windows read through a float4 cast (the round-3 form) instead of memcpy.
#define WS_LDU_CAST 1
#define WS_NS ws_f4cast
#define WS_API(name) name##_f4cast
#include "../qstep_ws.hip"
