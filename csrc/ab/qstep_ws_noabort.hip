// A/B build of csrc/qstep_ws.hip: ring waits without the sticky abort-word check.
#define WS_ABORT_WORD 0
#define WS_NS ws_noabort
#define WS_API(name) name##_noabort
#include "../qstep_ws.hip"
