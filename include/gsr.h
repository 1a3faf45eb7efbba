/*
 * gsr.h -- C ABI of the MI355X-native differentiable Gaussian rasterizer
 * (libgsr.so, built from 3d_gaussian_magic_change-segment_3dgs_amd/csrc/).
 *
 * Drop-in boundary for the reference's private extension module
 * `diff_gaussian_rasterization._C` (DGR/ext.cpp:15-19).  The Python package
 * diff_gaussian_rasterization (same directory tree) binds these symbols with
 * ctypes and keeps the reference's public API (GaussianRasterizationSettings,
 * GaussianRasterizer, rasterize_gaussians: DGR/diff_gaussian_rasterization/
 * __init__.py:21-236) unchanged.
 *
 * Conventions
 *   - Plain C: no C++ or HIP types.  `stream` is a hipStream_t passed as void*
 *     (torch.cuda.current_stream().cuda_stream); NULL = legacy default stream.
 *   - Every array pointer is a device pointer owned by the caller; the library
 *     never allocates device memory.  A NULL input pointer means "absent",
 *     mirroring the reference's empty-tensor convention (DGR/diff_gaussian_
 *     rasterization/__init__.py:208-221): exactly one of shs / colors_precomp,
 *     exactly one of (scales+rotations) / cov3D_precomp.  segments == NULL is
 *     read as zeros (the reference dereferences it unconditionally,
 *     forward.cu:369).
 *   - fp32 everywhere; images are planar CHW like the reference outputs
 *     (forward.cu:383-391).
 *   - Return value: 0 = success; non-zero = error, message in gsr_last_error()
 *     (thread-local).  settings->debug != 0 synchronises the stream after each
 *     stage and reports the first failing stage (reference CHECK_CUDA,
 *     auxiliary.h:166-173).
 *   - No global mutable device state: concurrent calls on distinct buffers and
 *     streams are safe (one process per GPU under torchrun).
 *   - Supersets of the reference's behaviour (no result the reference computes
 *     changes): settings->prefiltered = 1 never traps -- a Gaussian outside the
 *     frustum is culled as with prefiltered = 0 (the reference traps the whole
 *     kernel on one, auxiliary.h:156-160; its trainer always passes False);
 *     gradients are deterministic (no float atomics).
 */
#ifndef GSR_H_
#define GSR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define GSR_API __attribute__((visibility("default")))
#else
#define GSR_API
#endif

#define GSR_NUM_CHANNELS 3 /* reference config.h:15 */
#define GSR_NUM_CLASS 2    /* reference config.h:16 */
#define GSR_BLOCK_X 16     /* reference config.h:17 */
#define GSR_BLOCK_Y 16     /* reference config.h:18 */

/* Raster settings: the fields of GaussianRasterizationSettings
 * (DGR/diff_gaussian_rasterization/__init__.py:168-180) plus the problem sizes
 * the reference derives in RasterizeGaussiansCUDA (rasterize_points.cu:62-93). */
typedef struct gsr_settings {
    int P;                 /* number of Gaussians (means3D.shape[0]) */
    int D;                 /* active SH degree (sh_degree), 0..3 */
    int M;                 /* SH coefficients per channel (shs.shape[1]); 0 if shs absent */
    int W, H;              /* image_width, image_height */
    float tanfovx, tanfovy;
    float scale_modifier;
    int prefiltered;       /* accepted for API parity; culled points are never an error here */
    int debug;
    const float* bg;         /* device [3] */
    const float* viewmatrix; /* device [16], W2C^T row-major (scene/cameras.py:58) */
    const float* projmatrix; /* device [16], viewmatrix @ proj^T (scene/cameras.py:60) */
    const float* campos;     /* device [3] */
    /* Instances the binning buffer is laid out for; 0 = num_rendered.  gsr_forward with
     * binning_capacity = C > 0 (and a buffer of gsr_binning_bytes(C)) runs stage B before
     * num_rendered reaches the host; every later call on that buffer (gsr_backward,
     * gsr_backward_multiview, gsr_debug_copy) passes the same C.  For a buffer of exactly
     * gsr_binning_bytes(num_rendered), gsr_binning_capacity(size) is equivalent to 0. */
    int binning_capacity;
} gsr_settings;

/* Per-Gaussian inputs (device pointers, NULL = absent). */
typedef struct gsr_inputs {
    const float* means3D;        /* [P,3] */
    const float* shs;            /* [P,M,3] */
    const float* colors_precomp; /* [P,3] */
    const float* segments;       /* [P,2] */
    const float* opacities;      /* [P,1] (activated) */
    const float* scales;         /* [P,3] (activated) */
    const float* rotations;      /* [P,4] wxyz, normalised by the caller */
    const float* cov3D_precomp;  /* [P,6] upper triangle */
} gsr_inputs;

/* Gradient outputs of gsr_backward (device pointers; NULL = not wanted).
 * Every element of a non-NULL array is written (no pre-zeroing needed).
 * Replaces the zero-initialised tensors of rasterize_points.cu:166-177. */
typedef struct gsr_grads {
    float* dmeans2D;   /* [P,3]  NDC-space screen gradient, z = 0 */
    float* dcolors;    /* [P,3]  (grad of colors_precomp) */
    float* dopacity;   /* [P,1] */
    float* dmeans3D;   /* [P,3] */
    float* dcov3D;     /* [P,6]  (grad of cov3D_precomp) */
    float* dsh;        /* [P,M,3]; coefficients >= (D+1)^2 are written as 0 */
    float* dscales;    /* [P,3] */
    float* drot;       /* [P,4] */
    float* dsegments;  /* [P,2] */
} gsr_grads;

/* ---- size queries: the three byte buffers of the reference
 * (GeometryState / BinningState / ImageState, rasterizer_impl.h:29-73).  The
 * layout is private to the library and identical between forward and backward
 * for the same arguments. */
GSR_API size_t gsr_geom_bytes(int P);
GSR_API size_t gsr_binning_bytes(int num_rendered);
/* largest C with gsr_binning_bytes(C) <= bytes (-1 if none): the layout capacity of a binning
 * buffer of that size (settings.binning_capacity) */
GSR_API int gsr_binning_capacity(size_t bytes);
/* image-state buffer of a W x H view (ImageState, rasterizer_impl.cu:173-179).  Besides the
 * reference's ranges and n_contrib it holds the heavy-first tile schedule and, per 16x16 tile,
 * the forward's list-segment checkpoint for the backward (9 floats per pixel, 36 B): about
 * 88 MB in all at 1920 x 1080, 349 MB at 3840 x 2160, allocated whether or not a tile is deep enough
 * to use it; a multi-view forward keeps one per view until its backward. */
GSR_API size_t gsr_img_bytes(int W, int H);
/* scratch needed by gsr_backward (per-instance gradient records) */
GSR_API size_t gsr_backward_scratch_bytes(int num_rendered);

/* ---- forward, stage A: preprocess (projection, covariance, SH), depth order,
 * per-Gaussian tile counts and their prefix sum; copies num_rendered to the
 * host (the reference's single host sync, rasterizer_impl.cu:284-285).
 * Replaces Rasterizer::forward lines :226-289.  radii: device int32 [P]. */
GSR_API int gsr_forward_geometry(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii,
                         void* stream, int* num_rendered);

/* ---- forward, stage B: key duplication, tile sort, tile ranges and the tile
 * blend.  Replaces Rasterizer::forward lines :291-343 (duplicateWithKeys,
 * SortPairs, identifyTileRanges, renderCUDA).  Outputs: out_color [3,H,W],
 * out_depth [1,H,W], out_alpha [1,H,W] (= sum of alpha*T, forward.cu:386),
 * out_segment [2,H,W]. */
GSR_API int gsr_forward_render(const gsr_settings* s, const gsr_inputs* in, void* geom, void* binning,
                       void* img, int num_rendered, float* out_color, float* out_depth,
                       float* out_alpha, float* out_segment, void* stream);

/* ---- forward, both stages in one call (Rasterizer::forward, rasterizer_impl.cu:
 * 198-344): stage A, the num_rendered sync, then stage B straight from C when the
 * caller's binning buffer (binning_bytes, e.g. a guess from the previous view) holds
 * gsr_binning_bytes(num_rendered) -- no host-language round trip sits between the
 * sync and the render launches.  With s->binning_capacity = C > 0 and binning_bytes >=
 * gsr_binning_bytes(C), stage B is launched right behind stage A, before num_rendered
 * reaches the host (its kernels read it on the device and write nothing past C); the
 * host waits only afterwards.  If num_rendered turns out > C, stage B's outputs are void
 * and GSR_NEED_BINNING is returned.  Returns 0 (rendered), GSR_NEED_BINNING (stage A done,
 * *num_rendered set, nothing rendered: call gsr_forward_render with a buffer of
 * gsr_binning_bytes(*num_rendered)), or another nonzero error (gsr_last_error). */
#define GSR_NEED_BINNING 2
GSR_API int gsr_forward(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii, void* binning,
                        size_t binning_bytes, void* img, float* out_color, float* out_depth, float* out_alpha,
                        float* out_segment, void* stream, int* num_rendered);

/* ---- deferred forward (a multi-view batch): gsr_forward's speculative path (requires
 * s->binning_capacity = C > 0 and binning_bytes >= gsr_binning_bytes(C)) split in two.
 * gsr_forward_deferred launches stage A and stage B and returns at once with *ticket; the
 * host can launch the next views meanwhile (gsr_forward waits for num_rendered before it
 * returns, which gates the host's next launches on this view's binning).
 * gsr_forward_wait(ticket, the same s, geom and stream) then waits for num_rendered:
 * 0 (rendered), GSR_NEED_BINNING (num_rendered > C: stage B's outputs are void; call
 * gsr_forward_render with a buffer of gsr_binning_bytes(*num_rendered)), or an error.
 * Each host thread may hold up to GSR_MAX_DEFERRED tickets; every ticket must be waited
 * for (once).  No counterpart in the reference (rasterize_points.cu:35-125 renders one
 * view per call and syncs inside it). */
#define GSR_MAX_DEFERRED 16
GSR_API int gsr_forward_deferred(const gsr_settings* s, const gsr_inputs* in, void* geom, int* radii,
                                 void* binning, size_t binning_bytes, void* img, float* out_color,
                                 float* out_depth, float* out_alpha, float* out_segment, void* stream,
                                 int* ticket);
GSR_API int gsr_forward_wait(int ticket, const gsr_settings* s, const void* geom, void* stream,
                             int* num_rendered);

/* ---- backward.  Replaces Rasterizer::backward (rasterizer_impl.cu:348-458) /
 * RasterizeGaussiansBackwardCUDA (rasterize_points.cu:127-221).  dL_d* are the
 * upstream image gradients (same shapes as the forward outputs); alpha is the
 * forward's out_alpha; scratch has gsr_backward_scratch_bytes(num_rendered).
 * Contract: `in` must name the same colour source as the forward of this geom buffer
 * (shs, or colors_precomp) with the same tensors.  The forward stores the SH direction
 * Jacobian in geom only when it evaluated SH itself; a backward given shs after a
 * forward with colors_precomp would read that field uninitialised: libgsr records each
 * geom buffer's colour source at its forward and fails such a call (nonzero return,
 * gsr_last_error) instead.  (The reference recomputes it from shs; the Python layer always
 * passes the forward's inputs.) */
GSR_API int gsr_backward(const gsr_settings* s, const gsr_inputs* in, const int* radii, void* geom,
                 void* binning, void* img, int num_rendered, const float* alpha,
                 const float* dL_dcolor, const float* dL_dsegment, const float* dL_ddepth,
                 const float* dL_dalpha, void* scratch, const gsr_grads* grads, void* stream);

/* ---- multi-view backward: the parameter gradients of B views of the same
 * Gaussians, SUMMED over the views, in one call (the data-parallel trainer's
 * per-step batch).  Each view is a completed gsr_forward_* call with
 * its own settings (camera / image size; P, D and M must be equal) and upstream
 * gradients.  Equivalent to calling gsr_backward per view and adding the results
 * (tests/test_gpu_multiview.py), but the per-Gaussian part reads the shared
 * inputs (means, scales, rotations, SH rows) and writes the parameter gradients
 * once per batch instead of once per view.  dmeans2D stays per view (the
 * densification statistics are per view).  grads->dmeans2D is ignored. */
#define GSR_MAX_VIEWS 16
typedef struct gsr_view_state {
    const gsr_settings* s;
    const int* radii;
    void* geom;
    void* binning;
    void* img;
    int num_rendered;
    const float* alpha;
    const float* dL_dcolor;
    const float* dL_dsegment;
    const float* dL_ddepth;
    const float* dL_dalpha;
    void* scratch;    /* gsr_backward_scratch_bytes(num_rendered) */
    float* dmeans2D;  /* [P,3] this view's screen-space gradient, or NULL */
} gsr_view_state;
GSR_API size_t gsr_multiview_scratch_bytes(int P, int B);
GSR_API int gsr_backward_multiview(int B, const gsr_view_state* views, const gsr_inputs* in, void* mv_scratch,
                                   const gsr_grads* grads, void* stream);
/* ---- view-parallel exchange of the SH gradient.  For one view
 * the SH-coefficient gradient is the outer product basis(dir) x dRGB
 * (backward.cu:46-110): 48 floats per Gaussian determined by 3 (the clamped
 * colour gradient) and the camera centre.  A data-parallel trainer therefore
 * exchanges each view's dRGB rows (all-gather, 12 B per Gaussian and view) instead
 * of all-reducing dsh (192 B per Gaussian), and every rank rebuilds the summed dsh
 * locally with gsr_sh_backward.  The SH direction term of dmeans3D (dRGB . d(rgb)/d(dir),
 * backward.cu:54-111) is added by each rank for its own views inside the multi-view
 * backward, from the direction Jacobian each view's forward stored (36 B per Gaussian),
 * so dmeans3D is complete before it is all-reduced and the rebuild reads no SH row.
 *
 * gsr_sh_rows_floats(P): floats of one view's rows: dRGB [P,3], then the view's
 * camera centre (x, y, z, 0) at float offset roundup(3P, 64).
 *
 * gsr_backward_multiview_deferred_sh: gsr_backward_multiview (shs required) that
 * writes the B views' rows to sh_rows [B][gsr_sh_rows_floats(P)] (16-B aligned)
 * and leaves grads->dsh unwritten; all other gradients, dmeans3D included, are
 * complete (summed over the B views).
 *
 * gsr_sh_backward: for V views' rows (in order; every rank sums in the same order,
 * so all ranks get identical bits), writes dsh [P,M,3] = sum_v basis_v x dRGB_v
 * (coefficients >= (D+1)^2 written as 0).  Reads means3D and the rows only: shs and
 * dmeans3D are accepted for ABI compatibility and not used (shs may be NULL).  Run on
 * the all-gathered rows, the result equals the all-reduce of the complete dsh. */
GSR_API size_t gsr_sh_rows_floats(int P);
/* gsr_backward_deferred_sh: gsr_backward (shs required) that writes this view's rows to
 * sh_rows [gsr_sh_rows_floats(P)] (16-B aligned) instead of grads->dsh (left unwritten);
 * every other gradient, dmeans3D included, is complete.  One view per rank and step needs
 * no multi-view call: this is the single-view backward with 12 B of rows written in place
 * of the 192-B dsh rows. */
GSR_API int gsr_backward_deferred_sh(const gsr_settings* s, const gsr_inputs* in, const int* radii, void* geom,
                                     void* binning, void* img, int num_rendered, const float* alpha,
                                     const float* dL_dcolor, const float* dL_dsegment, const float* dL_ddepth,
                                     const float* dL_dalpha, void* scratch, const gsr_grads* grads, float* sh_rows,
                                     void* stream);
GSR_API int gsr_backward_multiview_deferred_sh(int B, const gsr_view_state* views, const gsr_inputs* in,
                                               float* sh_rows, const gsr_grads* grads, void* stream);
GSR_API int gsr_sh_backward(int V, int P, int D, int M, const float* shs, const float* means3D,
                            const float* sh_rows, float* dsh, float* dmeans3D, void* stream);

/* ---- native data-parallel exchange over RCCL (csrc/dp.hip).  The collectives of the
 * view-parallel trainer issued from C: one call orders the library's
 * communication stream after the caller's stream, issues the collectives as one RCCL group (and,
 * for the SH exchange, the dsh rebuild behind them) and returns a ticket; gsr_dp_wait(ticket,
 * stream) orders a stream after all of it.  A ticket stays valid for 16 later exchanges.
 * librccl is loaded at the first gsr_dp_get_unique_id / gsr_dp_init.  The communicator is the
 * library's own: rank 0 calls gsr_dp_get_unique_id (gsr_dp_unique_id_bytes() bytes), the caller
 * broadcasts them (e.g. torch.distributed), and every rank calls gsr_dp_init on its device.
 * gsr_dp_allreduce: in-place float sum of buf [n] over the ranks.
 * gsr_dp_sh_exchange: the SH exchange of one step (gsr_sh_backward above): sums the arena's
 * dmeans3D block and its [dopacity .. bucket end) blocks (include/gsr_train.h layout for P, M, C),
 * all-gathers each rank's views_per_rank views of rows [gsr_sh_rows_floats(P)] into rows_all
 * [world][views_per_rank][...] and rebuilds the arena's dsh block from them.  The caller keeps
 * arena, rows, rows_all and means3D alive and unread until it has waited on the ticket.
 * Both return the ticket (>= 0) or -1 (gsr_last_error()). */
GSR_API size_t gsr_dp_unique_id_bytes(void);
GSR_API int gsr_dp_get_unique_id(void* out);
GSR_API int gsr_dp_init(const void* unique_id, int world, int rank);
GSR_API int gsr_dp_world(void);  /* 0 before gsr_dp_init / after gsr_dp_finalize */
GSR_API int gsr_dp_finalize(void);
GSR_API int gsr_dp_allreduce(float* buf, size_t n, void* stream);
GSR_API int gsr_dp_sh_exchange(int P, int D, int M, int C, const float* means3D, int views_per_rank, float* arena,
                               const float* rows, float* rows_all, void* stream);
GSR_API int gsr_dp_wait(int ticket, void* stream);

/* ---- frustum visibility: present[i] = (view-space z > 0.2).  Replaces
 * markVisible (rasterize_points.cu:223-242, rasterizer_impl.cu:54-66). */
GSR_API int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/* ---- inspection hook for parity tests: copies one private intermediate of a
 * forward call into dst (device memory; stream-ordered).  Names and element
 * types: "tiles_touched" u32[P], "rec" f32[P,16] ({x,y,conic.xyz,opacity,depth,
 * seg0,r,g,b,seg1,0...}), "clamped" u8[P], "order" u32[P] (depth order),
 * "goff" u32[P] (the Gaussian's first record slot inside its block of 256 Gaussians: slots are
 * numbered in Gaussian-index order), "bbase" u32[ceil(P/256)] (the slots before each block),
 * "point_list" u32[I], "slot_vals" u32[I] (the radix binning's instance slots: -1 with an
 * error when the row binning -- the default for grids up to 255 x 255 tiles -- is active, as it
 * writes none), "ranges" u32[T,2],
 * "n_contrib_tiles" u32[T,256] (tile-major, in the forward's 8x8-quadrant layout:
 * entry k*64+l of tile (tx, ty) is pixel (16*tx + 8*(k&1) + (l&7), 16*ty + 8*(k>>1) + (l>>3)),
 * k = 0..3 the quadrant, l = 0..63 the lane), "written" u8[I] (after a backward: 1 at
 * every instance slot the render backward stored a gradient record for), "tile_order" u32[]
 * (the heavy-first tile order followed by the render schedule words).  Returns the byte count
 * copied (0 when the buffer holding the field is NULL), or -1; with dst = NULL, the byte count
 * a copy would take, without touching the device (callers size dst with it). */
GSR_API long long gsr_debug_copy(const char* name, int P, int W, int H, int num_rendered, int binning_capacity,
                                 void* geom, void* binning, void* img, void* dst, void* stream);

/* ---- live stage timing (bench/profiling): gsr_timing_enable(mask) brackets every
 * stage i with (mask >> i) & 1 set (mask -1 = all, 0 = off) by hipEvents recorded
 * on the caller's stream; no host synchronisation is added.  Each bracket costs a
 * few microseconds of stream time, so time only the stages needed.
 * gsr_timing_collect() waits for the recorded events,
 * accumulates per-stage milliseconds and launch counts into ms[i] / counts[i]
 * (arrays of gsr_num_stages() entries), and clears the pending list. */
#define GSR_STAGE_PREPROCESS 0
#define GSR_STAGE_DEPTH_SORT 1
#define GSR_STAGE_SCAN 2
#define GSR_STAGE_DUPLICATE 3
#define GSR_STAGE_TILE_SORT 4
#define GSR_STAGE_RANGES 5
#define GSR_STAGE_RENDER_FWD 6
#define GSR_STAGE_RENDER_BWD 7
#define GSR_STAGE_GAUSSIAN_BWD 8
GSR_API int gsr_num_stages(void);
GSR_API const char* gsr_stage_name(int stage);
GSR_API void gsr_timing_enable(int stage_mask);
GSR_API int gsr_timing_collect(double* ms, long long* counts);

/* HBM streaming-copy reference for the roofline (not part of the reference's interface):
 * copies `bytes` (a multiple of 16) from src to dst with `per_thread` (1, 2 or 4) float4 per
 * thread, non-temporal loads and stores, on `stream`.  bench.py times it with events to
 * report the achievable HBM rate of the box beside the 8 TB/s spec. */
GSR_API int gsr_stream_copy(const void* src, void* dst, size_t bytes, int per_thread, void* stream);

/* Thread-local message of the last failing call ("" if none). */
GSR_API const char* gsr_last_error(void);

/* Library version string (build identification). */
GSR_API const char* gsr_version(void);
/* ---- tuning / test hook (process-wide, not thread-safe against concurrent calls):
 * "sort_lookback_max": radix sorts of at most this many keys use the single-launch
 * look-back passes, larger ones the histogram-table passes (default 4194304; 0 forces the
 * table passes for every sort).  "sort_grouped" (0/1, default 1): key-only sorts of at most
 * 1024 tiles (4M keys, e.g. the depth sort) take the grouped look-back passes.
 * "rows_binning" (0/1, default 1), "speculate" (0/1, default 1), "split_fwd_bucket" /
 * "split4_fwd_bucket" (forward tiles with n >= 2^(B-1) instances on two / four waves; defaults
 * 8 / 0 = off), "split_bwd_depth" (backward two-wave tiles; default 0 = off); a negative value
 * restores a default.  Results are identical either way.  "bwd_ckpt" (list position, rounded up
 * to a multiple of 64; default 256, 0 = off): the forward checkpoints each pixel's replay state
 * there and the backward replays tiles deeper than it + 64 as two independent list segments
 * (render.hip publish_depth); gradients then differ from the unsegmented ones in fp32 rounding
 * (within the parity bounds) and colour / depth / segment outputs by a few ulps; it applies only
 * with split_bwd_depth = 0 and is read by the forward (the backward follows the forward's choice).
 * "mv_streams" (0/1, default 1): the multi-view backward's odd views on a second stream.
 * Returns 0, or non-zero for an unknown name. */
GSR_API int gsr_set_option(const char* name, long long value);

#ifdef __cplusplus
}
#endif

#endif /* GSR_H_ */
