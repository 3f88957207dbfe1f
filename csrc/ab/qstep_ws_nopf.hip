// Timing build of csrc/qstep_ws.hip (wrong results; never used for training): no price-window loads in
// the tile loop (every tile reuses the first tile's windows) -- prices the HBM latency the loop exposes.
// st_qstep_ws_launch_nopf (engine.step_variant = "nopf" with step_kernel "ws").
#define WS_NOPF 1
#define WS_NS ws_nopf
#define WS_API(name) name##_nopf
#include "../qstep_ws.hip"
