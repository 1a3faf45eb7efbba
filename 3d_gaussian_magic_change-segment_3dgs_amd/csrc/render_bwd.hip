// render_bwd.hip -- the render backward kernels (render.hip's GSR_RENDER_PART 2) as their own
// translation unit, so that the Makefile can build them with the max-ILP machine scheduler:
// k_render_bwd1 347-349 us against 351 with the default strategy, which costs the forward
// 16 us (profiles/round4_sched_strategy.txt).
#if !(defined(GSR_WAVE_TRACE) || defined(GSR_STATS))  // diagnostic builds: render.hip holds both parts
#define GSR_RENDER_PART 2
#include "render.hip"
#endif
