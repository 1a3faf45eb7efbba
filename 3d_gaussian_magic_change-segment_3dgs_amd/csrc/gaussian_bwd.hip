// gaussian_bwd.hip -- k_gaussian_backward (preprocess.hip's GSR_PRE_PART 2) as its own
// translation unit, so that the Makefile can build it with the iterative-ILP machine
// scheduler: 117.4-117.7 us against 120.7-120.9 with the default strategy
// (profiles/round4_sched_strategy.txt).
#define GSR_PRE_PART 2
#include "preprocess.hip"
