// Timing build of csrc/qstep_ws.hip: the gradient waves hand every ring slot back without computing
// (wrong gradients; never used for training) -- measures how fast the data waves run on their own.
// st_qstep_ws_launch_gskip (engine.step_variant = "gskip" with step_kernel "ws").
#define WS_GSKIP 1
#define WS_NS ws_gskip
#define WS_API(name) name##_gskip
#include "../qstep_ws.hip"
