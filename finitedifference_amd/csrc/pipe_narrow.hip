// pipe_narrow.hip -- the narrow-tile instantiations (W = 8, 16) of the pipe
// kernel (pipe.hip), compiled as their own unit with the default machine
// scheduler: with the narrow steady-edge blocks it keeps fewer scalars live
// (fewer reloads of spilled SGPRs) and runs the 1024^2 9-mu sweep 3.5 %
// faster, while max-ilp stays 0.9 % ahead on the wide 4096^2 kernel
// (profiles/r02/sched/).
#define BURG_PIPE_NARROW_TU 1
#include "pipe.hip"
