// Timing build of csrc/qstep_ws.hip: the prologue (bf16 weight images gathered into LDS) runs twice --
// prices the per-launch prologue.  st_qstep_ws_launch_pro2 (engine.step_variant = "pro2").
#define WS_PROLOGUE_REPS 2
#define WS_NS ws_pro2
#define WS_API(name) name##_pro2
#include "../qstep_ws.hip"
