// A/B build of csrc/qstep_ws.hip (correct results): WS_FIL with 8 VALU per layer-1 MFMA pair.
// st_qstep_ws_launch_fil8 (engine.step_variant = "fil8").
#define WS_FIL 1
#define WS_FILV 8
#define WS_NS ws_fil8
#define WS_API(name) name##_fil8
#include "../qstep_ws.hip"
