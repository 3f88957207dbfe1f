// timing build: csrc/qstep_pipe.hip with s_memtime stamps (tools/stamp_pipe.py); same results
#define PIPE_STAMPS 1
#define PIPE_NS pipe_stamps
#define PIPE_API(name) name##_stamps
#include "qstep_pipe.hip"
