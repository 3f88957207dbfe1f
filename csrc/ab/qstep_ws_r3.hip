// A/B reference: the round-3 production ws kernel, verbatim (csrc/ab/qstep_ws_r3.inc), as
// st_qstep_ws_launch_r3 -- so a change to csrc/qstep_ws.hip is timed against it on the same box.
#define WS_NS ws_r3
#define WS_API(name) name##_r3
#include "qstep_ws_r3.inc"
