// Tuning build of csrc/qstep_ws.hip: every price window read from replica 0 of the bank with 4-byte-aligned
// (not 16-byte-aligned) dwordx4 loads -- does the bank need its 4 alignment replicas?
// st_qstep_ws_launch_unal (engine.step_variant = "unal" with step_kernel "ws").
#define WS_UNAL 1
#define WS_NS ws_unal
#define WS_API(name) name##_unal
#include "qstep_ws.hip"
