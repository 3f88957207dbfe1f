// Tuning build of csrc/qstep_ws.hip: the next tile's price windows are issued right after this tile's
// features (a whole tile of HBM latency hidden, 63 more VGPRs live through the layers).
// st_qstep_ws_launch_pfe (engine.step_variant = "pfe" with step_kernel "ws").
#define WS_PF_POS 2
#define WS_NS ws_pfe
#define WS_API(name) name##_pfe
#include "qstep_ws.hip"
