// A/B build of csrc/qstep_ws.hip (correct results): WS_FIL with 6 VALU per layer-1 MFMA pair.
// st_qstep_ws_launch_fil6 (engine.step_variant = "fil6").
#define WS_FIL 1
#define WS_FILV 6
#define WS_NS ws_fil6
#define WS_API(name) name##_fil6
#include "../qstep_ws.hip"
