// pipe_narrow.hip -- the narrow-tile instantiations (W = 8, 16) of the pipe
// kernel (pipe.hip), compiled as their own unit (the two width classes were
// tuned with different machine schedulers in round 2; both use max-ilp since
// the narrow blocks grew to 8 diagonals, Makefile).
#define BURG_PIPE_NARROW_TU 1
#include "pipe.hip"
