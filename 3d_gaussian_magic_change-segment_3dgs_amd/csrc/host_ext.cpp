// host_ext.cpp -- the host side of the drop-in rasterizer in C++ (torch extension "gsr_host").
//
// Replaces the per-call host work of RasterizeGaussiansCUDA / RasterizeGaussiansBackwardCUDA
// (DGR/rasterize_points.cu:35-221): argument checks, output / buffer allocation and the
// libgsr calls (include/gsr.h).  diff_gaussian_rasterization/_C.py keeps the same work in
// Python over ctypes; when this module is built (__graft_entry__.build()) the single-view
// forward and backward go through it instead, because the Python version costs ~120 us of
// host time per view (profiles/round6_*_host_overhead.txt) -- enough to make small views
// host-bound.  Same semantics and error messages as _C.py: float32 inputs, CPU tensors moved
// to the device of means3D, re-allocation of misaligned inputs, the binning-capacity guess
// passed in by the caller (speculative stage B, gsr_forward), one gradient arena with the
// data-parallel bucket first.  The drop-in rasterize_gaussians() goes one step further through
// `rasterize`: the autograd function itself is C++ (RasterizeFn below), so a training step
// crosses into Python only at the caller's own code.  No compute here: every kernel is libgsr's.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "gsr.h"
#include "gsr_train.h"

namespace {

constexpr int ARENA_ALIGN = 64;  // gsr_train.h GSR_ARENA_ALIGN (floats)

// Host time spent inside libgsr's calls (launches and the forward's num_rendered wait), so that
// tools/host_overhead.py can separate the binding's own host time from them (lib_ns()).
std::atomic<long long> g_lib_ns{0};
struct LibTimer {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~LibTimer() {
        g_lib_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
};

void check(int rc) {
    if (rc) throw std::runtime_error(gsr_last_error());
}

bool present(const c10::optional<at::Tensor>& t) { return t.has_value() && t->defined() && t->numel() > 0; }

// _C.py _dev_f32: contiguous fp32 on `dev`, re-allocated if not `align`-byte aligned; empty -> undefined
at::Tensor dev_f32(const c10::optional<at::Tensor>& t, const at::Device& dev, const char* name, int align = 4) {
    if (!present(t)) return at::Tensor();
    at::Tensor u = *t;
    if (u.scalar_type() != at::kFloat)
        throw std::runtime_error(std::string(name) + " must be a float32 tensor (got " +
                                 std::string(c10::toString(u.scalar_type())) + ")");
    if (u.device() != dev) {
        if (!u.device().is_cpu())
            throw std::runtime_error(std::string(name) + " is on " + u.device().str() + ", expected " + dev.str());
        u = u.to(dev);
    }
    u = u.contiguous();
    if (reinterpret_cast<uintptr_t>(u.data_ptr()) % align) u = u.clone();
    return u;
}

const float* fptr(const at::Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }

// PyTorch-ROCm calls its HIP devices "cuda": the guard and the stream are the masquerading ones
// (torch.cuda.current_stream() of the current device)
void* cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

gsr_settings make_settings(int P, int D, int M, int W, int H, double tanx, double tany, double scale_modifier,
                           bool prefiltered, bool debug, const at::Tensor& bg, const at::Tensor& view,
                           const at::Tensor& proj, const at::Tensor& campos) {
    gsr_settings s{};
    s.P = P; s.D = D; s.M = M; s.W = W; s.H = H;
    s.tanfovx = (float)tanx; s.tanfovy = (float)tany; s.scale_modifier = (float)scale_modifier;
    s.prefiltered = prefiltered ? 1 : 0; s.debug = debug ? 1 : 0;
    s.bg = fptr(bg); s.viewmatrix = fptr(view); s.projmatrix = fptr(proj); s.campos = fptr(campos);
    s.binning_capacity = 0;
    return s;
}

int capacity_of(size_t bytes) { return bytes ? std::max(0, gsr_binning_capacity(bytes)) : 0; }

// A zero-filled [shape] tensor without memory traffic: one cached zero per device, expanded
// (_C.py _zeros; the reference returns torch::zeros, rasterize_points.cu:166-177).
at::Tensor zeros_view(const at::Device& dev, at::IntArrayRef shape) {
    // never destroyed: freeing device memory from a static destructor could run after the HIP
    // runtime has shut down at process exit
    static std::mutex mu;
    static auto* z = new std::vector<at::Tensor>(64);
    const int i = dev.index() < 0 ? 0 : dev.index() % 64;
    std::lock_guard<std::mutex> lk(mu);
    at::Tensor& t = (*z)[i];
    if (!t.defined() || t.device() != dev) t = at::zeros({}, at::TensorOptions().dtype(at::kFloat).device(dev));
    return t.expand(shape);
}

long long now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Deferred-SH sinks (diff_gaussian_rasterization.defer_sh_gradients): their count, kept by the
// Python context manager, and the Python function that runs a single-view backward through the
// active sink.  A backward of the autograd route that finds a sink active (and SH coefficients)
// hands its arguments to that function, as _RasterizeGaussians.backward would.
std::atomic<int> g_sinks{0};
py::object* g_sink_backward = nullptr;  // never destroyed (see zeros_view)

// Host-time stamps of the autograd route (tools/host_overhead.py): per call the entry time, the
// time inside libgsr and the exit time, steady_clock ns (CLOCK_MONOTONIC, as time.perf_counter_ns).
std::atomic<bool> g_stamps_on{false};
std::mutex g_stamp_mu;
std::vector<std::array<long long, 4>> g_stamps;  // kind (0 forward, 1 backward), t_in, lib_ns, t_out
void stamp(int kind, long long t_in, long long lib) {
    if (!g_stamps_on.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> lk(g_stamp_mu);
    g_stamps.push_back({kind, t_in, lib, now_ns()});
}

}  // namespace

// RasterizeGaussiansCUDA (rasterize_points.cu:35-125) with the caller's binning-capacity guess
// `cap` (0 = none): (num_rendered, color, depth, segment, alpha, radii, geom, binning, img).
using FwdOut = std::tuple<int64_t, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>;
using BwdOut = std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor>;

FwdOut rasterize_gaussians(const c10::optional<at::Tensor>& background, const at::Tensor& means3D,
                              const c10::optional<at::Tensor>& colors, const c10::optional<at::Tensor>& segments,
                              const c10::optional<at::Tensor>& opacity, const c10::optional<at::Tensor>& scales,
                              const c10::optional<at::Tensor>& rotations, double scale_modifier,
                              const c10::optional<at::Tensor>& cov3D_precomp,
                              const c10::optional<at::Tensor>& viewmatrix,
                              const c10::optional<at::Tensor>& projmatrix, double tan_fovx, double tan_fovy,
                              int64_t image_height, int64_t image_width, const c10::optional<at::Tensor>& sh,
                              int64_t degree, const c10::optional<at::Tensor>& campos, bool prefiltered, bool debug,
                              int64_t cap) {
    if (means3D.dim() != 2 || means3D.size(1) != 3) throw std::runtime_error("means3D must have dimensions (num_points, 3)");
    const int P = (int)means3D.size(0), H = (int)image_height, W = (int)image_width;
    const at::Device dev = means3D.device();
    if (!dev.is_cuda())
        throw std::runtime_error("gsr rasterizer: means3D must be a GPU tensor (the HIP path has no CPU fallback)");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(dev);
    const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    const auto u8 = at::TensorOptions().dtype(at::kByte).device(dev);
    if (P == 0) {  // the reference leaves the zero-filled outputs untouched (rasterize_points.cu:87)
        at::Tensor e = at::empty({0}, u8);
        return FwdOut(0, at::zeros({GSR_NUM_CHANNELS, H, W}, f32), at::zeros({1, H, W}, f32),
                              at::zeros({GSR_NUM_CLASS, H, W}, f32), at::zeros({1, H, W}, f32),
                              at::zeros({0}, f32.dtype(at::kInt)), e, at::empty({0}, u8), at::empty({0}, u8));
    }
    const at::Tensor m = dev_f32(means3D, dev, "means3D"), sh_ = dev_f32(sh, dev, "sh"),
                     col = dev_f32(colors, dev, "colors_precomp"), seg = dev_f32(segments, dev, "segments", 8);
    if (seg.defined() && (seg.dim() != 2 || seg.size(1) != GSR_NUM_CLASS || seg.size(0) != P))
        throw std::runtime_error("segments must have shape (num_points, 2) (reference config.h:16 NUM_CLASS)");
    const at::Tensor op = dev_f32(opacity, dev, "opacities"), sc = dev_f32(scales, dev, "scales"),
                     rot = dev_f32(rotations, dev, "rotations", 16), cov = dev_f32(cov3D_precomp, dev, "cov3D_precomp"),
                     bg = dev_f32(background, dev, "bg"), view = dev_f32(viewmatrix, dev, "viewmatrix"),
                     proj = dev_f32(projmatrix, dev, "projmatrix"), cp = dev_f32(campos, dev, "campos");
    const int M = sh_.defined() ? (int)sh_.size(1) : 0;
    gsr_settings s = make_settings(P, (int)degree, M, W, H, tan_fovx, tan_fovy, scale_modifier, prefiltered, debug, bg,
                                   view, proj, cp);
    const gsr_inputs in{fptr(m), fptr(sh_), fptr(col), fptr(seg), fptr(op), fptr(sc), fptr(rot), fptr(cov)};
    void* st = cur_stream();
    at::Tensor geom = at::empty({(int64_t)gsr_geom_bytes(P)}, u8);
    at::Tensor img = at::empty({(int64_t)gsr_img_bytes(W, H)}, u8);
    at::Tensor radii = at::empty({P}, f32.dtype(at::kInt));
    at::Tensor color = at::empty({GSR_NUM_CHANNELS, H, W}, f32), depth = at::empty({1, H, W}, f32);
    at::Tensor alpha = at::empty({1, H, W}, f32), segment = at::empty({GSR_NUM_CLASS, H, W}, f32);
    at::Tensor binning = cap > 0 ? at::empty({(int64_t)gsr_binning_bytes((int)cap)}, u8) : at::Tensor();
    s.binning_capacity = binning.defined() ? capacity_of((size_t)binning.numel()) : 0;
    int nr = 0;
    LibTimer lt;
    int rc = gsr_forward(&s, &in, geom.data_ptr(), radii.data_ptr<int>(), binning.defined() ? binning.data_ptr() : nullptr,
                         binning.defined() ? (size_t)binning.numel() : 0, img.data_ptr(), color.data_ptr<float>(),
                         depth.data_ptr<float>(), alpha.data_ptr<float>(), segment.data_ptr<float>(), st, &nr);
    if (rc == GSR_NEED_BINNING) {  // no guess, or too small: stage B with the exact size
        binning = at::empty({(int64_t)gsr_binning_bytes(nr)}, u8);
        s.binning_capacity = capacity_of((size_t)binning.numel());
        rc = gsr_forward_render(&s, &in, geom.data_ptr(), binning.data_ptr(), img.data_ptr(), nr,
                                color.data_ptr<float>(), depth.data_ptr<float>(), alpha.data_ptr<float>(),
                                segment.data_ptr<float>(), st);
    }
    check(rc);
    if (!binning.defined()) binning = at::empty({0}, u8);
    // the reference's return order (rasterize_points.cu:124)
    return FwdOut(nr, color, depth, segment, alpha, radii, geom, binning, img);
}

// RasterizeGaussiansBackwardCUDA (rasterize_points.cu:127-221): one gradient arena, the
// data-parallel bucket [dmeans3D | dsh | dopacity | dscales | drot | dsegments] first
// (_C.py grad_arena_layout); gradients of absent inputs are stride-0 zero views.
BwdOut rasterize_gaussians_backward(
    const c10::optional<at::Tensor>& background, const at::Tensor& means3D, const at::Tensor& radii,
    const c10::optional<at::Tensor>& colors, const c10::optional<at::Tensor>& segments,
    const c10::optional<at::Tensor>& scales, const c10::optional<at::Tensor>& rotations, double scale_modifier,
    const c10::optional<at::Tensor>& cov3D_precomp, const c10::optional<at::Tensor>& viewmatrix,
    const c10::optional<at::Tensor>& projmatrix, double tan_fovx, double tan_fovy,
    const c10::optional<at::Tensor>& dL_dout_color, const c10::optional<at::Tensor>& dL_dout_segment,
    const c10::optional<at::Tensor>& dL_dout_depth, const c10::optional<at::Tensor>& dL_dout_alpha,
    const c10::optional<at::Tensor>& sh, int64_t degree, const c10::optional<at::Tensor>& campos,
    const at::Tensor& geomBuffer, int64_t R, const at::Tensor& binningBuffer, const at::Tensor& imageBuffer,
    const at::Tensor& alpha, bool debug) {
    const int P = (int)means3D.size(0);
    const at::Tensor* shaped = nullptr;
    for (const auto* t : {&dL_dout_color, &dL_dout_segment, &dL_dout_depth, &dL_dout_alpha})
        if (t->has_value() && (*t)->defined()) { shaped = &**t; break; }
    if (!shaped) shaped = &alpha;
    const int H = (int)shaped->size(-2), W = (int)shaped->size(-1);
    const at::Device dev = means3D.device();
    c10::hip::HIPGuardMasqueradingAsCUDA guard(dev);
    const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    const at::Tensor m = dev_f32(means3D, dev, "means3D"), sh_ = dev_f32(sh, dev, "sh"),
                     col = dev_f32(colors, dev, "colors_precomp"), seg = dev_f32(segments, dev, "segments", 8),
                     sc = dev_f32(scales, dev, "scales"), rot = dev_f32(rotations, dev, "rotations", 16),
                     cov = dev_f32(cov3D_precomp, dev, "cov3D_precomp");
    const int M = sh_.defined() ? (int)sh_.size(1) : 0;
    // grad arena (_C.py grad_arena_layout): 6 bucket blocks, then dmeans2D, dcolors, dcov3D
    long long off[7];
    gsr_arena_layout(P, M, GSR_NUM_CLASS, off);
    const long long o2d = off[6];
    const long long ocol = o2d + (3LL * P + ARENA_ALIGN - 1) / ARENA_ALIGN * ARENA_ALIGN;
    const long long ocov = ocol + (3LL * P + ARENA_ALIGN - 1) / ARENA_ALIGN * ARENA_ALIGN;
    const long long total = ocov + (6LL * P + ARENA_ALIGN - 1) / ARENA_ALIGN * ARENA_ALIGN;
    at::Tensor arena = at::empty({total}, f32);
    auto view_of = [&](long long o, int k, std::initializer_list<int64_t> shape) {
        return arena.narrow(0, o, (int64_t)k * P).view(shape);
    };
    at::Tensor dmeans3D = view_of(off[0], 3, {P, 3}), dsh = view_of(off[1], 3 * M, {P, M, 3}),
               dopacity = view_of(off[2], 1, {P, 1}), dscales = view_of(off[3], 3, {P, 3}),
               drot = view_of(off[4], 4, {P, 4}), dsegments = view_of(off[5], GSR_NUM_CLASS, {P, GSR_NUM_CLASS}),
               dmeans2D = view_of(o2d, 3, {P, 3}), dcolors = view_of(ocol, 3, {P, 3}), dcov3D = view_of(ocov, 6, {P, 6});
    if (P == 0) {
        arena.zero_();
        return BwdOut(dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot, dsegments);
    }
    const at::Tensor bg = dev_f32(background, dev, "bg"), view = dev_f32(viewmatrix, dev, "viewmatrix"),
                     proj = dev_f32(projmatrix, dev, "projmatrix"), cp = dev_f32(campos, dev, "campos");
    gsr_settings s = make_settings(P, (int)degree, M, W, H, tan_fovx, tan_fovy, scale_modifier, false, debug, bg, view,
                                   proj, cp);
    s.binning_capacity = capacity_of((size_t)binningBuffer.numel());
    const gsr_inputs in{fptr(m), fptr(sh_), fptr(col), fptr(seg), nullptr, fptr(sc), fptr(rot), fptr(cov)};
    const char* names[4] = {"dL_dcolor", "dL_dsegment", "dL_ddepth", "dL_dalpha"};
    const int chans[4] = {GSR_NUM_CHANNELS, GSR_NUM_CLASS, 1, 1};
    const c10::optional<at::Tensor>* ins[4] = {&dL_dout_color, &dL_dout_segment, &dL_dout_depth, &dL_dout_alpha};
    at::Tensor ups[4];
    for (int i = 0; i < 4; ++i) {
        ups[i] = dev_f32(*ins[i], dev, names[i]);
        if (!ups[i].defined()) ups[i] = at::zeros({chans[i], H, W}, f32);  // a gradient autograd did not materialise
    }
    const at::Tensor alpha_ = dev_f32(alpha, dev, "alpha");
    const at::Tensor radii_ = radii.contiguous();
    const int Ri = (int)R;
    at::Tensor scratch = at::empty({(int64_t)gsr_backward_scratch_bytes(Ri)}, f32.dtype(at::kByte));
    gsr_grads g{};
    g.dmeans2D = dmeans2D.data_ptr<float>();
    g.dopacity = dopacity.data_ptr<float>();
    g.dmeans3D = dmeans3D.data_ptr<float>();
    g.dcolors = col.defined() ? dcolors.data_ptr<float>() : nullptr;
    g.dcov3D = cov.defined() ? dcov3D.data_ptr<float>() : nullptr;
    g.dsh = (sh_.defined() && M > 0) ? dsh.data_ptr<float>() : nullptr;
    g.dscales = sc.defined() ? dscales.data_ptr<float>() : nullptr;
    g.drot = sc.defined() ? drot.data_ptr<float>() : nullptr;
    g.dsegments = dsegments.data_ptr<float>();
    LibTimer lt;
    check(gsr_backward(&s, &in, radii_.data_ptr<int>(), geomBuffer.data_ptr(),
                       binningBuffer.numel() ? binningBuffer.data_ptr() : nullptr, imageBuffer.data_ptr(), Ri,
                       alpha_.data_ptr<float>(), ups[0].data_ptr<float>(), ups[1].data_ptr<float>(),
                       ups[2].data_ptr<float>(), ups[3].data_ptr<float>(), Ri > 0 ? scratch.data_ptr() : nullptr, &g,
                       cur_stream()));
    return BwdOut(dmeans2D, col.defined() ? dcolors : zeros_view(dev, {P, 3}), dopacity, dmeans3D,
                          cov.defined() ? dcov3D : zeros_view(dev, {P, 6}), sh_.defined() ? dsh : zeros_view(dev, {P, 0, 3}),
                          sc.defined() ? dscales : zeros_view(dev, {P, 3}), sc.defined() ? drot : zeros_view(dev, {P, 4}),
                          seg.defined() ? dsegments : zeros_view(dev, {P, GSR_NUM_CLASS}));
}

// _RasterizeGaussians (DGR/diff_gaussian_rasterization/__init__.py:46-166) as a C++ autograd
// function: the same saved state, the same outputs (color, radii, depth, alpha, segment), radii
// non-differentiable, unmaterialised output gradients read as zeros, and the same gradient
// hand-back (_finish_grads: nothing for an input that needs none, a real zero tensor where an
// input that needs one got a stride-0 placeholder).  The Python function costs ~100 us of host
// time per view in autograd's Python hops (profiles/round6_*_host_overhead.txt); it still serves
// debug mode (snapshot dumps) and forwards run inside defer_sh_gradients.
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

struct RasterizeFn : public torch::autograd::Function<RasterizeFn> {
    static variable_list forward(AutogradContext* ctx, const at::Tensor& means3D, const at::Tensor& means2D,
                                 const at::Tensor& sh, const at::Tensor& colors, const at::Tensor& segments,
                                 const at::Tensor& opacities, const at::Tensor& scales, const at::Tensor& rotations,
                                 const at::Tensor& cov3D, const at::Tensor& bg, const at::Tensor& view,
                                 const at::Tensor& proj, const at::Tensor& campos, double scale_modifier, double tanx,
                                 double tany, int64_t H, int64_t W, int64_t degree, bool prefiltered, int64_t cap,
                                 int64_t* num_rendered) {
        (void)means2D;  // the screen-space gradient's carrier: it receives dmeans2D
        const long long t_in = now_ns(), l0 = g_lib_ns.load();
        auto [nr, color, depth, segment, alpha, radii, geom, binning, img] =
            rasterize_gaussians(bg, means3D, colors, segments, opacities, scales, rotations, scale_modifier, cov3D,
                                view, proj, tanx, tany, H, W, sh, degree, campos, prefiltered, false, cap);
        *num_rendered = nr;
        ctx->saved_data["num_rendered"] = nr;
        ctx->saved_data["scale_modifier"] = scale_modifier;
        ctx->saved_data["tanfovx"] = tanx;
        ctx->saved_data["tanfovy"] = tany;
        ctx->saved_data["sh_degree"] = degree;
        ctx->saved_data["geom"] = geom;
        ctx->saved_data["binning"] = binning;
        ctx->saved_data["img"] = img;
        // the settings' tensors as the Python function keeps them (ctx.raster_settings): referenced,
        // not version-checked; the Gaussian tensors and the outputs as its save_for_backward
        ctx->saved_data["bg"] = bg;
        ctx->saved_data["viewmatrix"] = view;
        ctx->saved_data["projmatrix"] = proj;
        ctx->saved_data["campos"] = campos;
        ctx->save_for_backward({colors, segments, means3D, scales, rotations, cov3D, radii, sh, alpha});
        ctx->mark_non_differentiable({radii});
        ctx->set_materialize_grads(false);
        stamp(0, t_in, g_lib_ns.load() - l0);
        return {color, radii, depth, alpha, segment};
    }

    static variable_list backward(AutogradContext* ctx, variable_list go) {
        const long long t_in = now_ns(), l0 = g_lib_ns.load();
        const auto sv = ctx->get_saved_variables();
        const at::Tensor &colors = sv[0], &segments = sv[1], &means3D = sv[2], &scales = sv[3], &rotations = sv[4],
                         &cov3D = sv[5], &radii = sv[6], &sh = sv[7], &alpha = sv[8];
        const at::Tensor bg = ctx->saved_data["bg"].toTensor(), view = ctx->saved_data["viewmatrix"].toTensor(),
                         proj = ctx->saved_data["projmatrix"].toTensor(), campos = ctx->saved_data["campos"].toTensor();
        const int64_t nr = ctx->saved_data["num_rendered"].toInt(), degree = ctx->saved_data["sh_degree"].toInt();
        const double sm = ctx->saved_data["scale_modifier"].toDouble(), tx = ctx->saved_data["tanfovx"].toDouble(),
                     ty = ctx->saved_data["tanfovy"].toDouble();
        const at::Tensor geom = ctx->saved_data["geom"].toTensor(), binning = ctx->saved_data["binning"].toTensor(),
                         img = ctx->saved_data["img"].toTensor();
        // output gradients in the order of the outputs: color, radii, depth, alpha, segment
        at::Tensor g[9];
        if (g_sinks.load() > 0 && sh.numel() > 0 && g_sink_backward) {
            py::gil_scoped_acquire gil;
            auto opt = [](const at::Tensor& t) { return t.defined() ? py::cast(t) : py::none(); };
            py::tuple r = (*g_sink_backward)(bg, means3D, radii, colors, segments, scales, rotations, sm, cov3D, view,
                                             proj, tx, ty, opt(go[0]), opt(go[4]), opt(go[2]), opt(go[3]), sh, degree,
                                             campos, geom, nr, binning, img, alpha);
            for (int i = 0; i < 9; ++i) g[i] = r[i].is_none() ? at::Tensor() : r[i].cast<at::Tensor>();
        } else {
            auto o = rasterize_gaussians_backward(bg, means3D, radii, colors, segments, scales, rotations, sm, cov3D,
                                                  view, proj, tx, ty, go[0], go[4], go[2], go[3], sh, degree, campos,
                                                  geom, nr, binning, img, alpha, false);
            std::tie(g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8]) = o;
        }
        // (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot, dsegments) -> input order
        const at::Tensor grads[9] = {g[3], g[0], g[5], g[1], g[8], g[2], g[6], g[7], g[4]};
        variable_list out(22);  // one per forward argument; none for the settings and the scalars
        for (int i = 0; i < 9; ++i) {
            const at::Tensor& t = grads[i];
            if (!t.defined() || !ctx->needs_input_grad(i)) continue;
            bool placeholder = false;
            if (t.numel() > 0)
                for (int64_t st : t.strides()) placeholder |= st == 0;
            out[i] = placeholder ? at::zeros(t.sizes(), t.options()) : t;
        }
        stamp(1, t_in, g_lib_ns.load() - l0);
        return out;
    }
};

// (color, radii, depth, alpha, segment, num_rendered); `cap`: the caller's binning-capacity guess
// (_C.py _guess, which num_rendered then feeds)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, int64_t> rasterize(
    const at::Tensor& means3D, const at::Tensor& means2D, const at::Tensor& sh, const at::Tensor& colors,
    const at::Tensor& segments, const at::Tensor& opacities, const at::Tensor& scales, const at::Tensor& rotations,
    const at::Tensor& cov3D, const at::Tensor& bg, const at::Tensor& view, const at::Tensor& proj,
    const at::Tensor& campos, double scale_modifier, double tanx, double tany, int64_t H, int64_t W, int64_t degree,
    bool prefiltered, int64_t cap) {
    int64_t nr = 0;
    auto o = RasterizeFn::apply(means3D, means2D, sh, colors, segments, opacities, scales, rotations, cov3D, bg, view,
                                proj, campos, scale_modifier, tanx, tany, H, W, degree, prefiltered, cap, &nr);
    return {o[0], o[1], o[2], o[3], o[4], nr};
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, mod) {  // the single-view entry points of DGR/ext.cpp:15-19
    // the GIL is released for the whole call, as ctypes does for foreign calls: the forward
    // waits for num_rendered inside gsr_forward
    mod.def("rasterize_gaussians", &rasterize_gaussians, py::call_guard<py::gil_scoped_release>());
    mod.def("rasterize_gaussians_backward", &rasterize_gaussians_backward, py::call_guard<py::gil_scoped_release>());
    mod.def("rasterize", &rasterize, py::call_guard<py::gil_scoped_release>());
    mod.def("set_sinks", [](int n) { g_sinks.store(n); });
    mod.def("set_sink_backward", [](py::object f) {
        if (!g_sink_backward) g_sink_backward = new py::object();
        *g_sink_backward = std::move(f);
    });
    mod.def("stamps", [](bool on) {  // enables / disables the stamps; returns and clears those taken
        std::lock_guard<std::mutex> lk(g_stamp_mu);
        g_stamps_on.store(on);
        std::vector<std::array<long long, 4>> r;
        r.swap(g_stamps);
        return r;
    });
    mod.def("version", []() { return std::string(gsr_version()); });
    mod.def("lib_ns", []() { return (long long)g_lib_ns.load(); });
}
