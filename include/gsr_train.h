/*
 * gsr_train.h -- C ABI of the training-step kernels around the rasterizer
 * (SURVEY.md s8f): parameter activations, the fused Adam step, densification
 * statistics and densify/prune compaction, over one "Gaussian arena".
 * Same library (libgsr.so) and conventions as gsr.h: plain C, caller-owned
 * device pointers, void* stream = hipStream_t, 0 = success / non-zero = error
 * with the message in gsr_last_error().
 *
 * The reference keeps each Gaussian attribute as its own nn.Parameter with its
 * own torch.optim.Adam param group (scene/gaussian_model.py:139-181) and
 * activates them with torch ops every iteration (:100-127).  Here every
 * per-Gaussian fp32 attribute lives in ONE buffer with a fixed block layout,
 * so a training step touches each byte once:
 *
 *   block  attribute (reference name)             floats / Gaussian
 *   0      xyz            (_xyz)                  3
 *   1      features       (_features_dc | _rest)  3*M   ([P,M,3]; coefficient 0 = f_dc)
 *   2      opacity        (_opacity, raw)         1
 *   3      scaling        (_scaling, raw = log)   3
 *   4      rotation       (_rotation, raw wxyz)   4
 *   5      segment        (_segment, raw)         C
 *
 * Each block starts at a multiple of GSR_ARENA_ALIGN floats.  Parameters, their
 * gradients and both Adam moments use the same layout, and so does the first
 * part of the rasterizer's gradient arena (blocks 0..5 = the data-parallel
 * all-reduce bucket [dmeans3D | dsh | dopacity | dscales | drot | dsegments]).
 *
 * The "activated" buffer holds what the rasterizer consumes for blocks 2..5:
 * sigmoid(opacity), exp(scaling), normalize(rotation), sigmoid(segment)
 * (gaussian_model.py:34-43,100-127), in blocks a0..a3 with the same alignment
 * rule; xyz and features are consumed raw.
 */
#ifndef GSR_TRAIN_H_
#define GSR_TRAIN_H_
#include <stddef.h>
#include <stdint.h>
#include "gsr.h"
#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ARENA_ALIGN 64  /* floats (256 B) */
#define GSR_ARENA_BLOCKS 6
#define GSR_ACT_BLOCKS 4

/* Block offsets (floats) of the parameter arena: off[0..5] = blocks 0..5,
 * off[6] = total floats.  Returns off[6]. */
GSR_API long long gsr_arena_layout(int P, int M, int C, long long* off);
/* Block offsets of the activated buffer: off[0..3] = opacity, scaling, rotation,
 * segment; off[4] = total floats.  Returns off[4]. */
GSR_API long long gsr_act_layout(int P, int C, long long* off);

/* Forward activations (replaces get_opacity / get_scaling / get_rotation /
 * get_segment, gaussian_model.py:100-127): act <- f(param) for blocks 2..5. */
GSR_API int gsr_activate(int P, int M, int C, const float* param, float* act, void* stream);

/* Backward of the activations, in place on the gradient arena's blocks 2..5:
 * d/d(raw) = d/d(activated) * f'(raw) (torch's exp / sigmoid / normalize
 * backward).  Blocks 0..1 pass through untouched. */
GSR_API int gsr_activation_backward(int P, int M, int C, const float* param, const float* act, float* grad,
                                    void* stream);

/* Adam hyper-parameters of one step, per reference param group
 * (gaussian_model.py:162-170 order: xyz, f_dc, f_rest, opacity, segment,
 * scaling, rotation).  step_size[g] = lr_g / (1 - beta1^t_g) and
 * bc2_sqrt[g] = sqrt(1 - beta2^t_g) are computed by the caller in double, as
 * torch.optim.Adam does (_multi_tensor_adam, capturable=False). */
#define GSR_ADAM_GROUPS 7
typedef struct gsr_adam_hyper {
    float beta1, beta2, eps;
    float one_minus_beta1, one_minus_beta2;  /* 1 - beta in double, then rounded (torch's lerp / addcmul weights) */
    float step_size[GSR_ADAM_GROUPS];
    float bc2_sqrt[GSR_ADAM_GROUPS];
    int skip[GSR_ADAM_GROUPS];  /* non-zero: leave the group untouched (grad None) */
} gsr_adam_hyper;

/* One Adam step over the whole arena (replaces gaussians.optimizer.step(),
 * train.py:185, with torch.optim.Adam(eps=1e-15), gaussian_model.py:172):
 *   m <- m + (1-b1)(g - m);  v <- b2 v + (1-b2) g^2;
 *   p <- p - step_size * m / (sqrt(v) / bc2_sqrt + eps)
 * If act is non-NULL, the activated values of the updated blocks 2..5 are
 * written too, so the next forward needs no activation pass. */
GSR_API int gsr_adam_step(int P, int M, int C, float* param, const float* grad, float* exp_avg,
                          float* exp_avg_sq, float* act, const gsr_adam_hyper* h, void* stream);

/* Densification statistics of one view (train.py:168-172,
 * gaussian_model.py:523-526).  A Gaussian is updated when filter[i] != 0 (the
 * reference's update_filter, a bool tensor) or, with filter == NULL, when
 * radii[i] > 0 (visibility_filter, gaussian_renderer/__init__.py:376):
 *   accum += |dmeans2D[i, :2]|;  denom += 1;
 *   max_radii2D = max(max_radii2D, radii)   (only if radii and max_radii2D are given).
 * dmeans2D is the rasterizer's [P,3] screen-space gradient. */
GSR_API int gsr_densify_stats(int P, const uint8_t* filter, const int* radii, const float* dmeans2D,
                              float* max_radii2D, float* grad_accum, float* denom, void* stream);

/* ---- densification and pruning (gaussian_model.py:386-521) as two calls around
 * one host sync (the reference syncs too: boolean-mask indexing).
 *
 * gsr_densify_plan classifies every Gaussian and counts the survivors:
 *   mode GSR_DENSIFY_AND_PRUNE  densify_and_prune(max_grad, min_opacity, extent,
 *                               max_screen_size) -- clone small / split large
 *                               Gaussians whose mean view-space gradient
 *                               (grad_accum / denom, NaN -> 0) >= max_grad, then
 *                               prune sigmoid(opacity) < min_opacity and, if
 *                               max_screen_size > 0, world-space size
 *                               > 0.1 * extent (the screen-size test reads
 *                               max_radii2D after densification_postfix reset it
 *                               to 0, as the reference does);
 *   mode GSR_PRUNE_MASK         prune_points(mask): drop mask[i] != 0;
 *   mode GSR_CLONE_ONLY         densify_and_clone(grads, max_grad, extent);
 *   mode GSR_SPLIT_ONLY         densify_and_split(grads, max_grad, extent, N).
 * counts (host int[4]) = {kept originals, kept clones, kept split children per
 * copy, split-selected Gaussians}; the new size is c0 + c1 + split_n * c2.
 * gsr_densify_apply then writes the new arenas in the reference's order
 * [kept originals | kept clones | children copy 0 | ... | copy N-1] (stable):
 * clones copy their source, children get xyz = R(q) (z * s) + xyz and
 * scaling = log(s / (0.8 N)) with s = exp(scaling) and z the caller's standard
 * normal draws [split_n * c3, 3] (the reference's torch.normal(0, s), which
 * draws z with normal_(0, 1) and multiplies by s).  New Gaussians get zero Adam
 * moments; kept ones keep theirs (cat_tensors_to_optimizer / _prune_optimizer).
 * ws holds gsr_densify_ws_bytes(P) bytes and carries the plan to the apply. */
#define GSR_DENSIFY_AND_PRUNE 0
#define GSR_PRUNE_MASK 1
#define GSR_CLONE_ONLY 2
#define GSR_SPLIT_ONLY 3
typedef struct gsr_densify_args {
    int mode;
    int split_n;             /* N of densify_and_split (2 in the reference) */
    float max_grad;          /* densify_grad_threshold */
    float min_opacity;
    float clone_max_scale;   /* percent_dense * scene_extent (computed in double, rounded) */
    float prune_max_scale;   /* 0.1 * extent */
    float max_screen_size;   /* <= 0: None */
    float split_divisor;     /* 0.8 * N (computed in double, rounded) */
} gsr_densify_args;
GSR_API size_t gsr_densify_ws_bytes(int P);
GSR_API int gsr_densify_plan(int P, int M, int C, const float* param, const float* act, const float* grad_accum,
                             const float* denom, const uint8_t* mask, const gsr_densify_args* a, void* ws,
                             int* counts, void* stream);
GSR_API int gsr_densify_apply(int P, int M, int C, const float* param, const float* act, const float* exp_avg,
                              const float* exp_avg_sq, const gsr_densify_args* a, const void* ws, const int* counts,
                              const float* normals, float* new_param, float* new_exp_avg, float* new_exp_avg_sq,
                              void* stream);

/* ---- PLY vertex rows <-> arena (save_ply / load_ply, gaussian_model.py:207-262 and
 * the multi-scene merge of visualizer.py:196-226).  `rows` is the file's vertex
 * block as float32 rows of row_floats columns, on the device.  col[k] names the row
 * column of arena float k of one Gaussian, k in arena order (xyz 3 | features 3M
 * as [M,3] | opacity | scaling 3 | rotation 4 | segment C), -1 = not in the file
 * (zero).  rows_to_arena writes Gaussians [dst, dst + n) of an arena sized for P
 * (so several files merge into one arena); arena_to_rows writes every column of
 * every row (columns no arena float maps to, e.g. the normals, become 0). */
#define GSR_PLY_MAX_COLS 128
GSR_API int gsr_ply_rows_to_arena(int n, int row_floats, const float* rows, const int* col, int P, int M, int C,
                                  int dst, float* param, void* stream);
GSR_API int gsr_arena_to_ply_rows(int P, int M, int C, const float* param, int row_floats, const int* col,
                                  float* rows, void* stream);

/* ---- distCUDA2 (submodules_local/simple-knn/simple_knn.cu:181-220, called at
 * gaussian_model.py:143): mean_dists[i] = mean squared distance of point i to its
 * 3 nearest other points (exact).  points: device [P,3]; ws: gsr_knn_ws_bytes(P). */
GSR_API size_t gsr_knn_ws_bytes(int P);
GSR_API int gsr_dist_knn3(int P, const float* points, float* mean_dists, void* ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_TRAIN_H_ */
