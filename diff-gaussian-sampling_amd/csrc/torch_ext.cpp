// torch_ext.cpp -- diff_gaussian_sampling._C: the reference's pybind surface (ext.cpp:19-32)
// mapped onto the C ABI of libdgs.so (include/dgs.h).
//
// Same function names, argument order and meaning, return arity and error behaviour as the
// reference host glue (sample_points.{h,cu}, aggregate_neighbors.{h,cu}):
//   * inputs are borrowed, made contiguous; wrong dtypes raise RuntimeError (the reference's
//     data<float>() check); P == 0 or N == 0 returns zero/empty results without launching;
//   * the tile grid of sample_points.cu:70-74 is computed on the device with torch's CUDA-path
//     arithmetic and read back at the binning's one host sync (dgs_preprocess_auto);
//   * opaque u8 buffers come back to Python and are handed back verbatim;
//   * everything runs on torch's current HIP stream; `debug` synchronises and checks after
//     every launch (auxiliary.h:33-40).
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <tuple>
#include <vector>

#include "dgs.h"
#include "dgs_volume.h"

namespace {

using torch::Tensor;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// Whether torch's current stream is being captured into a graph (torch.cuda.graph): the sample
// calls then enqueue kernels only (DGS_SAMPLE_GRAPH_CAPTURE) and keep no packed-row records.
bool capturing() {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(cur_stream(), &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}
const char *const kCaptureMsg =
    "under graph capture, means, conics and samples must be the tensors the binning was made from "
    "(unmodified since; a binning cannot be captured)";
dgs_stream_t as_dgs(hipStream_t s) { return reinterpret_cast<dgs_stream_t>(s); }

void check(int rc, const char *what) {
    if (rc != DGS_OK) throw std::runtime_error(std::string(what) + ": " + dgs_last_error());
}

Tensor f32(const Tensor &t, const char *name) {
    TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be a float32 tensor (got ",
                t.scalar_type(), ")");
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    return t.contiguous();
}

Tensor u8(const Tensor &t, const char *name) {
    TORCH_CHECK(t.scalar_type() == torch::kUInt8, name, " must be the uint8 buffer returned by preprocess");
    return t.contiguous();
}

struct AllocCtx {
    torch::Device device;
    Tensor bufs[8];
    std::vector<Tensor> scratch;
};

void *alloc_cb(void *vctx, int which, size_t bytes) {
    auto *ctx = static_cast<AllocCtx *>(vctx);
    try {
        Tensor t = torch::empty({(int64_t)bytes}, torch::TensorOptions().dtype(torch::kUInt8).device(ctx->device));
        void *p = t.data_ptr();
        if (which >= 0 && which < 8 && which != DGS_BUF_SCRATCH) ctx->bufs[which] = t;
        else ctx->scratch.push_back(t);
        return p;
    } catch (...) {
        return nullptr;
    }
}

Tensor empty_u8(const torch::Device &dev) {
    return torch::empty({0}, torch::TensorOptions().dtype(torch::kUInt8).device(dev));
}

using PreOut = std::tuple<int64_t, Tensor, Tensor, Tensor, Tensor, Tensor>;

// ---- per-step caches of the sampling calls (dgs_sample_options) ------------------------------
// A tensor's identity: its storage (weakly held), data pointer, element count and autograd
// version.  A tensor and its .detach() share storage and version counter, so they are the same
// here; every in-place op through either bumps the shared version.  Writes that bypass the
// counter (through .data, or raw pointers) are not seen: DGS_ALWAYS_VERIFY=1 or debug=True keep
// the device-side comparison for code that does that.
using WeakImpl = c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>;
using WeakStorage = c10::weak_intrusive_ptr<c10::StorageImpl>;
struct TKey {
    WeakStorage storage;
    const void *ptr;
    int64_t numel, version;
};
// Inference tensors (torch.inference_mode) have no version counter: calls on them keep no
// records and always take the device-side comparison (as do buffers made under inference mode).
bool trackable(std::initializer_list<const Tensor *> ts) {
    for (const Tensor *t : ts)
        if (t->is_inference()) return false;
    return true;
}
TKey tkey(const Tensor &t) {
    return {t.storage().getWeakStorageImpl(), t.data_ptr(), t.numel(), (int64_t)t._version()};
}
bool same(const TKey &k, const Tensor &t) {
    const auto sp = k.storage.lock();
    return sp && sp.get() == t.storage().unsafeGetStorageImpl() && k.ptr == t.data_ptr() && k.numel == t.numel() &&
           k.version == (int64_t)t._version();
}

bool always_verify() {
    static const bool on = [] {
        const char *e = std::getenv("DGS_ALWAYS_VERIFY");
        return e && e[0] && e[0] != '0';
    }();
    return on;
}

// What each binning was built from (preprocess): a forward / backward passing exactly those
// means / conics / samples needs no device-side comparison (DGS_SAMPLE_INPUTS_BINNED).
struct BinRecord {
    TKey gb, means, conics, samples;
};
// The workspace of a forward whose Gaussian rows a later call on the same binning, function
// mask and parameters reuses (DGS_SAMPLE_ROWS_VALID): the forward of a training step packs
// them, its backward uses them (one pack per step instead of two).
struct RowRecord {
    TKey gb, means, values, conics;
    int mask, C;
    Tensor work;
    hipStream_t stream;  // the stream that packed the rows: reused only on it (stream order)
};
std::mutex g_step_mu;
std::vector<BinRecord> g_bins;
std::vector<RowRecord> g_rows;

void bins_put(const Tensor &gb, const Tensor &means, const Tensor &conics, const Tensor &samples) {
    std::lock_guard<std::mutex> lk(g_step_mu);
    for (auto it = g_bins.begin(); it != g_bins.end();)
        if (it->gb.storage.expired() || it->gb.ptr == gb.data_ptr()) it = g_bins.erase(it);
        else ++it;
    if (!trackable({&gb, &means, &conics, &samples})) return;
    g_bins.push_back({tkey(gb), tkey(means), tkey(conics), tkey(samples)});
    if (g_bins.size() > 8) g_bins.erase(g_bins.begin());
}

bool inputs_binned(const Tensor &gb, const Tensor &means, const Tensor &conics, const Tensor &samples) {
    if (always_verify() || !trackable({&gb, &means, &conics, &samples})) return false;
    std::lock_guard<std::mutex> lk(g_step_mu);
    for (const auto &r : g_bins)
        if (same(r.gb, gb)) return same(r.means, means) && same(r.conics, conics) && same(r.samples, samples);
    return false;
}

// take = true: remove the record (a backward overwrites the rows).
bool rows_get(const Tensor &gb, int mask, int C, const Tensor &means, const Tensor &values, const Tensor &conics,
              size_t need, bool take, Tensor &work) {
    if (!trackable({&gb, &means, &values, &conics})) return false;
    const hipStream_t st = cur_stream();
    std::lock_guard<std::mutex> lk(g_step_mu);
    for (auto it = g_rows.begin(); it != g_rows.end(); ++it) {
        if (it->mask != mask || it->C != C || !same(it->gb, gb)) continue;
        const bool ok = it->stream == st && same(it->means, means) && same(it->values, values) &&
                        same(it->conics, conics) && (size_t)it->work.numel() >= need;
        if (ok) work = it->work;
        if (take || !ok) g_rows.erase(it);
        return ok;
    }
    return false;
}

void rows_put(const Tensor &gb, int mask, int C, const Tensor &means, const Tensor &values, const Tensor &conics,
              const Tensor &work) {
    std::lock_guard<std::mutex> lk(g_step_mu);
    for (auto it = g_rows.begin(); it != g_rows.end();)
        if (it->gb.storage.expired() || (it->mask == mask && it->gb.ptr == gb.data_ptr())) it = g_rows.erase(it);
        else ++it;
    if (!trackable({&gb, &means, &values, &conics})) return;
    // (the workspace was allocated on the current stream and is only reused on it: rows_get)
    g_rows.push_back({tkey(gb), tkey(means), tkey(values), tkey(conics), mask, C, work, cur_stream()});
    if (g_rows.size() > 4) g_rows.erase(g_rows.begin());  // (the per-function path of a fused call keeps one per function)
}

// The sample buffer of the last eager binnings per samples tensor (dgs_bin_options.samples_binned):
// a later binning of the same, unchanged samples copies its sample side instead of sorting the
// samples again (the training loop re-bins after every optimizer step; its points stay put).
struct SampleRecord {
    TKey samples;
    Tensor sb;
    hipStream_t stream;  // the binning's stream: copied from only on it (stream order)
};
std::vector<SampleRecord> g_samples;

Tensor samples_get(const Tensor &samples) {
    if (always_verify() || !trackable({&samples})) return Tensor();
    std::lock_guard<std::mutex> lk(g_step_mu);
    const hipStream_t st = cur_stream();
    for (const auto &r : g_samples)
        if (r.stream == st && same(r.samples, samples)) return r.sb;
    return Tensor();
}

void samples_put(const Tensor &samples, const Tensor &sb) {
    std::lock_guard<std::mutex> lk(g_step_mu);
    for (auto it = g_samples.begin(); it != g_samples.end();)
        if (it->samples.storage.expired() || same(it->samples, samples)) it = g_samples.erase(it);
        else ++it;
    if (!trackable({&samples}) || sb.numel() == 0) return;
    g_samples.push_back({tkey(samples), sb, cur_stream()});
    if (g_samples.size() > 2) g_samples.erase(g_samples.begin());  // (a train and a test set, say)
}

PreOut preprocess_impl(const Tensor &means_in, const Tensor &values_in, const Tensor &cov_in,
                       const Tensor &conics_in, const Tensor &samples_in, const std::vector<int> *grid_in,
                       const std::vector<float> *off_in, bool debug, const dgs_bin_options *opts_in = nullptr) {
    const Tensor means = f32(means_in, "means"), covs = f32(cov_in, "covariances");
    const Tensor conics = f32(conics_in, "conics"), samples = f32(samples_in, "samples");
    (void)values_in;
    const int P = (int)means.size(0), D = (int)means.size(-1), N = (int)samples.size(0);
    // (k_gauss_prep writes every radius when there is anything to bin; zeros otherwise)
    Tensor radii = P != 0 && N != 0 ? torch::empty({P}, means.options()) : torch::full({P}, 0, means.options());
    AllocCtx ctx{means.device()};
    for (int i = 0; i < 4; ++i) ctx.bufs[i] = empty_u8(means.device());
    int64_t rendered = 0;
    // the eager binnings (not the capturable one): the sample buffer of an earlier binning of
    // these samples, if they are unchanged since
    dgs_bin_options o{};
    if (opts_in) o = *opts_in;
    o.struct_size = sizeof(dgs_bin_options);
    const bool eager = o.capacity_E <= 0;
    Tensor prev_sb;
    if (eager && samples.data_ptr() == samples_in.data_ptr()) prev_sb = samples_get(samples_in);
    if (prev_sb.defined()) {
        o.samples_binned = prev_sb.data_ptr();
        o.samples_binned_bytes = (size_t)prev_sb.numel();
    }
    const dgs_bin_options *opts = &o;
    if (P != 0 && N != 0) {
        TORCH_CHECK(D == 1 || D == 2, "only D = 1 or D = 2 is supported (the reference leaves D = 3 undefined)");
        TORCH_CHECK(samples.size(-1) == D, "samples must have the same dimension as means");
        if (grid_in) {
            TORCH_CHECK((int)grid_in->size() == D && (int)off_in->size() == D, "grid/offset must have D entries");
            check(dgs_preprocess_ex(P, D, N, means.data_ptr<float>(), covs.data_ptr<float>(),
                                    conics.data_ptr<float>(), samples.data_ptr<float>(), grid_in->data(),
                                    off_in->data(), opts, radii.data_ptr<float>(), alloc_cb, &ctx, &rendered,
                                    as_dgs(cur_stream()), debug ? 1 : 0),
                  "preprocess_gaussians");
        } else {  // the grid of sample_points.cu:70-74 on the device: one host sync per call
            int grid[2];
            float off[2];
            check(dgs_preprocess_auto_ex(P, D, N, means.data_ptr<float>(), covs.data_ptr<float>(),
                                         conics.data_ptr<float>(), samples.data_ptr<float>(), opts,
                                         radii.data_ptr<float>(), alloc_cb, &ctx, &rendered, grid, off,
                                         as_dgs(cur_stream()), debug ? 1 : 0),
                  "preprocess_gaussians");
        }
    }
    if (ctx.bufs[DGS_BUF_BINNING].numel() > 0) bins_put(ctx.bufs[DGS_BUF_BINNING], means_in, conics_in, samples_in);
    // (the samples tensor as passed: a float32 contiguous one is its own binning input)
    if (eager && samples.data_ptr() == samples_in.data_ptr()) samples_put(samples_in, ctx.bufs[DGS_BUF_SAMPLE_BINNING]);
    return std::make_tuple(rendered, ctx.bufs[DGS_BUF_BINNING], ctx.bufs[DGS_BUF_SAMPLE_BINNING],
                           ctx.bufs[DGS_BUF_RANGES], ctx.bufs[DGS_BUF_SAMPLE_RANGES], radii);
}

// The graph-capturable binning (dgs_bin_options.capacity_E): the caller's
// grid / offset and capacities [E, Es, R] (binning_info of an earlier binning plus slack); no
// host sync, so it can be captured with torch.cuda.graph together with the sample calls.
// Returns (num_rendered int64[1] and status int32[1] on the device, binning buffers, ranges,
// radii); status != 0: the capacities were too small or the samples' grid changed (dgs.h).
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor>
PreprocessCapturableCUDA(const Tensor &means, const Tensor &values, const Tensor &covariances, const Tensor &conics,
                         const Tensor &samples, std::vector<int> grid, std::vector<float> offset,
                         std::vector<int64_t> capacity, const bool debug,
                         const c10::optional<Tensor> &status_in, const c10::optional<Tensor> &samples_binned) {
    TORCH_CHECK(capacity.size() == 3 && capacity[0] > 0 && capacity[2] > 0 && capacity[1] >= 0,
                "capacity must be [E > 0, Es >= 0, R > 0]");
    Tensor rdev = torch::zeros({1}, means.options().dtype(torch::kInt64));
    dgs_bin_options o{};
    o.struct_size = sizeof(dgs_bin_options);
    Tensor status;
    if (status_in.has_value() && status_in->defined()) {  // sticky: the caller's word, ORed into
        status = *status_in;
        TORCH_CHECK(status.is_cuda() && status.scalar_type() == torch::kInt32 && status.numel() == 1 &&
                        status.is_contiguous() && status.device() == means.device(),
                    "status must be a contiguous int32[1] tensor on the means' device");
        o.flags = DGS_BIN_STATUS_STICKY;
    } else {
        status = torch::zeros({1}, means.options().dtype(torch::kInt32));
    }
    if (samples_binned.has_value() && samples_binned->defined()) {  // fixed samples (the caller's word)
        TORCH_CHECK(samples_binned->scalar_type() == torch::kUInt8 && samples_binned->is_cuda() &&
                        samples_binned->is_contiguous(),
                    "samples_binned must be the sample_binning_buffer of an eager binning of these samples");
        o.samples_binned = samples_binned->data_ptr();
        o.samples_binned_bytes = (size_t)samples_binned->numel();
        o.flags |= DGS_BIN_SAMPLES_FIXED;
    }
    o.capacity_E = capacity[0];
    o.capacity_Es = std::min(capacity[1], capacity[0]);
    o.capacity_R = capacity[2];
    o.num_rendered_device = rdev.data_ptr<int64_t>();
    o.status_device = reinterpret_cast<uint32_t *>(status.data_ptr<int32_t>());
    PreOut r = preprocess_impl(means, values, covariances, conics, samples, &grid, &offset, debug, &o);
    return std::make_tuple(rdev, std::get<1>(r), std::get<2>(r), std::get<3>(r), std::get<4>(r), std::get<5>(r),
                           status);
}

// PreprocessCUDA (sample_points.h:20-27)
PreOut PreprocessCUDA(const Tensor &means, const Tensor &values, const Tensor &covariances,
                      const Tensor &conics, const Tensor &samples, const bool debug) {
    return preprocess_impl(means, values, covariances, conics, samples, nullptr, nullptr, debug);
}

// Sharded extension: the same with a caller-given (global) tile grid and offset.
PreOut PreprocessBoundedCUDA(const Tensor &means, const Tensor &values, const Tensor &covariances,
                             const Tensor &conics, const Tensor &samples, std::vector<int> grid,
                             std::vector<float> offset, const bool debug) {
    return preprocess_impl(means, values, covariances, conics, samples, &grid, &offset, debug);
}

// Spatially sharded ranks (distributed.SpatialShardedGaussianSampler): the global grid, only the
// Gaussians with present[g] != 0 (uint8/bool [P], or None = all), fine cells sized for the
// samples' own area (0 = the whole grid).
PreOut PreprocessShardedCUDA(const Tensor &means, const Tensor &values, const Tensor &covariances,
                             const Tensor &conics, const Tensor &samples, std::vector<int> grid,
                             std::vector<float> offset, const c10::optional<Tensor> &present_in,
                             const double sample_area, const bool debug) {
    dgs_bin_options o{};
    o.struct_size = sizeof(dgs_bin_options);
    Tensor present;
    if (present_in.has_value() && present_in->defined()) {
        TORCH_CHECK(present_in->scalar_type() == torch::kUInt8 || present_in->scalar_type() == torch::kBool,
                    "present must be a uint8 or bool tensor");
        TORCH_CHECK(present_in->is_cuda() && present_in->numel() == means.size(0), "present must be a GPU tensor of P");
        present = present_in->contiguous().view(torch::kUInt8);
        o.present = present.data_ptr<uint8_t>();
    }
    TORCH_CHECK(sample_area >= 0.0, "sample_area must be >= 0");
    o.sample_area = sample_area;
    return preprocess_impl(means, values, covariances, conics, samples, &grid, &offset, debug, &o);
}

std::vector<int64_t> out_shape(int fn, int64_t N, int64_t D, int64_t C) {
    std::vector<int64_t> shape{N};
    for (int k = 0; k < fn; ++k) shape.push_back(D);
    shape.push_back(C);
    return shape;
}

// The forward of every function of `mask` in one call (dgs_sample_forward_ex).  The call-time
// inputs are compared with the binned ones on the host (object identity + version counters,
// BinRecord) and, when any of means / values / conics requires a gradient, the workspace is
// sized for the backward and kept for it with its packed Gaussian rows (RowRecord).
void forward_mask(int mask, const Tensor &means_in, const Tensor &values_in, const Tensor &conics_in,
                  const Tensor &samples_in, const Tensor &binning_in, const Tensor &sbinning_in, float *const *outs,
                  bool debug) {
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    const Tensor conics = f32(conics_in, "conics"), samples = f32(samples_in, "samples");
    const int P = (int)means.size(0), D = (int)means.size(-1), N = (int)samples.size(0);
    const int C = (int)values.size(-1);
    if (P == 0 || N == 0) return;
    const Tensor gb = u8(binning_in, "binning_buffer"), sb = u8(sbinning_in, "sample_binning_buffer");
    dgs_sample_options o{};
    const bool cap = capturing();
    if (inputs_binned(binning_in, means_in, conics_in, samples_in)) o.flags |= DGS_SAMPLE_INPUTS_BINNED;
    else TORCH_CHECK(!cap, "sample_gaussians: ", kCaptureMsg);
    if (cap) o.flags |= DGS_SAMPLE_GRAPH_CAPTURE;
    const bool keep = !cap && (means_in.requires_grad() || values_in.requires_grad() || conics_in.requires_grad());
    const size_t ws = std::max(dgs_sample_workspace_size_multi(mask, P, D, N, C, 0),
                               keep ? dgs_sample_workspace_size_binned(mask, P, D, N, C, 1, gb.data_ptr(),
                                                                       (size_t)gb.numel(), sb.data_ptr(),
                                                                       (size_t)sb.numel())
                                    : (size_t)0);
    Tensor work;
    if (!cap && rows_get(binning_in, mask, C, means_in, values_in, conics_in, ws, false, work))
        o.flags |= DGS_SAMPLE_ROWS_VALID;
    else work = torch::empty({(int64_t)ws}, means.options().dtype(torch::kUInt8));
    check(dgs_sample_forward_ex(mask, P, D, N, C, means.data_ptr<float>(), values.data_ptr<float>(),
                                conics.data_ptr<float>(), samples.data_ptr<float>(), gb.data_ptr(), (size_t)gb.numel(),
                                sb.data_ptr(), (size_t)sb.numel(), outs, work.data_ptr(), (size_t)work.numel(), &o,
                                as_dgs(cur_stream()), debug ? 1 : 0),
          "sample_gaussians");
    if (keep && !(o.flags & DGS_SAMPLE_ROWS_VALID)) rows_put(binning_in, mask, C, means_in, values_in, conics_in, work);
}

Tensor sample_generic(int fn, const Tensor &means_in, const Tensor &values_in, const Tensor &conics_in,
                      const Tensor &samples_in, const Tensor &binning_in, const Tensor &sbinning_in,
                      bool debug) {
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    f32(conics_in, "conics");
    const Tensor samples = f32(samples_in, "samples");
    const int D = (int)means.size(-1);
    Tensor out = torch::full(out_shape(fn, samples.size(0), D, values.size(-1)), 0.0, means.options());
    float *outs[4] = {nullptr, nullptr, nullptr, nullptr};
    outs[fn] = out.data_ptr<float>();
    forward_mask(1 << fn, means_in, values_in, conics_in, samples_in, binning_in, sbinning_in, outs, debug);
    return out;
}

using Grads = std::tuple<Tensor, Tensor, Tensor>;

Grads backward_mask(int mask, const Tensor &means_in, const Tensor &values_in, const Tensor &conics_in,
                    const Tensor &samples_in, const float *const *dls, const Tensor &binning_in,
                    const Tensor &sbinning_in, bool debug) {
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    const Tensor conics = f32(conics_in, "conics"), samples = f32(samples_in, "samples");
    const int P = (int)means.size(0), D = (int)means.size(-1), N = (int)samples.size(0);
    const int C = (int)values.size(-1);
    // dgs_sample_backward_ex overwrites every gradient element; nothing to do -> zeros
    const auto alloc = [&](int64_t cols) {
        return N != 0 ? torch::empty({P, cols}, means.options()) : torch::zeros({P, cols}, means.options());
    };
    Tensor dmeans = alloc(D), dvalues = alloc(C), dconics = alloc(D * (D + 1) / 2);
    if (P != 0 && N != 0) {
        const Tensor gb = u8(binning_in, "binning_buffer"), sb = u8(sbinning_in, "sample_binning_buffer");
        dgs_sample_options o{};
        const bool cap = capturing();
        if (inputs_binned(binning_in, means_in, conics_in, samples_in)) o.flags |= DGS_SAMPLE_INPUTS_BINNED;
        else TORCH_CHECK(!cap, "sample_gaussians backward: ", kCaptureMsg);
        if (cap) o.flags |= DGS_SAMPLE_GRAPH_CAPTURE;
        // (the binned size: room for the slot sums where the binning wants them)
        const size_t ws = dgs_sample_workspace_size_binned(mask, P, D, N, C, 1, gb.data_ptr(), (size_t)gb.numel(),
                                                           sb.data_ptr(), (size_t)sb.numel());
        Tensor work;
        if (!cap && rows_get(binning_in, mask, C, means_in, values_in, conics_in, ws, true, work))
            o.flags |= DGS_SAMPLE_ROWS_VALID;
        else work = torch::empty({(int64_t)ws}, means.options().dtype(torch::kUInt8));
        check(dgs_sample_backward_ex(mask, P, D, N, C, means.data_ptr<float>(), values.data_ptr<float>(),
                                     conics.data_ptr<float>(), samples.data_ptr<float>(), dls, gb.data_ptr(),
                                     (size_t)gb.numel(), sb.data_ptr(), (size_t)sb.numel(), dmeans.data_ptr<float>(),
                                     dvalues.data_ptr<float>(), dconics.data_ptr<float>(), work.data_ptr(),
                                     (size_t)work.numel(), &o, as_dgs(cur_stream()), debug ? 1 : 0),
              "sample_gaussians_backward");
    }
    return std::make_tuple(dmeans, dvalues, dconics);
}

Grads sample_backward_generic(int fn, const Tensor &means_in, const Tensor &values_in,
                              const Tensor &conics_in, const Tensor &samples_in, const Tensor &dL_in,
                              const Tensor &binning_in, const Tensor &sbinning_in, bool debug) {
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    const Tensor samples = f32(samples_in, "samples");
    const int D = (int)means.size(-1);
    const int64_t N = samples.size(0), C = values.size(-1);
    Tensor dL;
    const float *dls[4] = {nullptr, nullptr, nullptr, nullptr};
    if (means.size(0) != 0 && N != 0) {
        dL = f32(dL_in, "dL_dout_values");
        int64_t K = 1;
        for (int k = 0; k < fn; ++k) K *= D;
        TORCH_CHECK(dL.numel() == N * K * C, "dL_dout has the wrong number of elements");
        dls[fn] = dL.data_ptr<float>();
    }
    return backward_mask(1 << fn, means_in, values_in, conics_in, samples_in, dls, binning_in, sbinning_in, debug);
}

#define DGS_FWD(NAME, FN)                                                                       \
    Tensor NAME(const Tensor &means, const Tensor &values, const Tensor &conics,                \
                const Tensor &samples, const int64_t num_rendered, const Tensor &binning_buffer, \
                const Tensor &sample_binning_buffer, const Tensor &ranges,                      \
                const Tensor &sample_ranges, const bool debug) {                                \
        (void)num_rendered; (void)ranges; (void)sample_ranges;                                  \
        return sample_generic(FN, means, values, conics, samples, binning_buffer,              \
                              sample_binning_buffer, debug);                                    \
    }
#define DGS_BWD(NAME, FN)                                                                       \
    Grads NAME(const Tensor &means, const Tensor &values, const Tensor &conics,                 \
               const Tensor &samples, const int64_t num_rendered, const Tensor &dL_dout_values, \
               const Tensor &binning_buffer, const Tensor &sample_binning_buffer,               \
               const Tensor &ranges, const Tensor &sample_ranges, const bool debug) {           \
        (void)num_rendered; (void)ranges; (void)sample_ranges;                                  \
        return sample_backward_generic(FN, means, values, conics, samples, dL_dout_values,     \
                                       binning_buffer, sample_binning_buffer, debug);           \
    }

// sample_points.h:29-131
DGS_FWD(SampleGaussiansCUDA, DGS_GAUSSIAN)
DGS_FWD(SampleGaussiansDerivativeCUDA, DGS_DERIVATIVE)
DGS_FWD(SampleGaussiansLaplacianCUDA, DGS_LAPLACIAN)
DGS_FWD(SampleGaussiansThirdCUDA, DGS_THIRD)
DGS_BWD(SampleGaussiansBackwardCUDA, DGS_GAUSSIAN)
DGS_BWD(SampleGaussiansDerivativeBackwardCUDA, DGS_DERIVATIVE)
DGS_BWD(SampleGaussiansLaplacianBackwardCUDA, DGS_LAPLACIAN)
DGS_BWD(SampleGaussiansThirdBackwardCUDA, DGS_THIRD)

// Fused functions (dgs_sample_{forward,backward}_multi): `functions` holds
// distinct codes 0..3; the outputs come back in that order.  Several functions at D = 2,
// C = 1 share one traversal of the pairs; otherwise the per-function kernels run in turn (on
// the GPU) and the backward adds their gradients.
static int function_mask(const std::vector<int64_t> &functions) {
    int mask = 0;
    for (int64_t f : functions) {
        TORCH_CHECK(f >= 0 && f <= 3, "sampling function codes are 0..3");
        TORCH_CHECK(!(mask & (1 << f)), "each sampling function may appear once");
        mask |= 1 << f;
    }
    TORCH_CHECK(mask != 0, "no sampling function given");
    return mask;
}

std::vector<Tensor> SampleGaussiansMulti(const std::vector<int64_t> &functions, const Tensor &means_in,
                                         const Tensor &values_in, const Tensor &conics_in,
                                         const Tensor &samples_in, const Tensor &binning_in,
                                         const Tensor &sbinning_in, const bool debug) {
    const int mask = function_mask(functions);
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    f32(conics_in, "conics");
    const Tensor samples = f32(samples_in, "samples");
    const int D = (int)means.size(-1), C = (int)values.size(-1);
    std::vector<Tensor> outs;
    if (functions.size() == 1 || D != 2 || C != 1) {
        for (int64_t f : functions)
            outs.push_back(sample_generic((int)f, means_in, values_in, conics_in, samples_in, binning_in, sbinning_in,
                                          debug));
        return outs;
    }
    float *ptr[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int64_t f : functions) {
        outs.push_back(torch::full(out_shape((int)f, samples.size(0), D, C), 0.0, means.options()));
        ptr[f] = outs.back().data_ptr<float>();
    }
    forward_mask(mask, means_in, values_in, conics_in, samples_in, binning_in, sbinning_in, ptr, debug);
    return outs;
}

Grads SampleGaussiansMultiBackward(const std::vector<int64_t> &functions, const Tensor &means_in,
                                   const Tensor &values_in, const Tensor &conics_in,
                                   const Tensor &samples_in, const std::vector<Tensor> &dLs_in,
                                   const Tensor &binning_in, const Tensor &sbinning_in, const bool debug) {
    const int mask = function_mask(functions);
    TORCH_CHECK(dLs_in.size() == functions.size(), "one dL_dout per sampling function");
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    const Tensor samples = f32(samples_in, "samples");
    const int P = (int)means.size(0), D = (int)means.size(-1), N = (int)samples.size(0);
    const int C = (int)values.size(-1);
    if (functions.size() == 1 || D != 2 || C != 1) {
        Grads g = sample_backward_generic((int)functions[0], means_in, values_in, conics_in, samples_in, dLs_in[0],
                                          binning_in, sbinning_in, debug);
        for (size_t i = 1; i < functions.size(); ++i) {
            Grads h = sample_backward_generic((int)functions[i], means_in, values_in, conics_in, samples_in,
                                              dLs_in[i], binning_in, sbinning_in, debug);
            std::get<0>(g).add_(std::get<0>(h));
            std::get<1>(g).add_(std::get<1>(h));
            std::get<2>(g).add_(std::get<2>(h));
        }
        return g;
    }
    std::vector<Tensor> dLs;
    const float *ptr[4] = {nullptr, nullptr, nullptr, nullptr};
    if (P != 0 && N != 0)
        for (size_t i = 0; i < functions.size(); ++i) {
            const int f = (int)functions[i];
            dLs.push_back(f32(dLs_in[i], "dL_dout_values"));
            TORCH_CHECK(dLs.back().numel() == (int64_t)N * (1 << f), "dL_dout has the wrong number of elements");
            ptr[f] = dLs.back().data_ptr<float>();
        }
    return backward_mask(mask, means_in, values_in, conics_in, samples_in, ptr, binning_in, sbinning_in, debug);
}

// Diagnostics: (W_cand, W_live) over the pairs the forward evaluates.
std::tuple<int64_t, int64_t> CountPairs(const Tensor &means_in, const Tensor &conics_in,
                                        const Tensor &samples_in, const Tensor &binning_in,
                                        const Tensor &sbinning_in, double thr) {
    const Tensor means = f32(means_in, "means"), conics = f32(conics_in, "conics");
    const Tensor samples = f32(samples_in, "samples");
    const int P = (int)means.size(0), D = (int)means.size(-1), N = (int)samples.size(0);
    int64_t counts[2] = {0, 0};
    if (P != 0 && N != 0) {
        const Tensor gb = u8(binning_in, "binning_buffer"), sb = u8(sbinning_in, "sample_binning_buffer");
        const size_t ws = dgs_sample_workspace_size(0, P, D, N, 1, 0) + 256;
        Tensor work = torch::empty({(int64_t)ws}, means.options().dtype(torch::kUInt8));
        check(dgs_count_pairs(P, D, N, means.data_ptr<float>(), conics.data_ptr<float>(),
                              samples.data_ptr<float>(), gb.data_ptr(), (size_t)gb.numel(),
                              sb.data_ptr(), (size_t)sb.numel(), (float)thr, counts, work.data_ptr(),
                              ws, as_dgs(cur_stream())),
              "count_pairs");
    }
    return std::make_tuple(counts[0], counts[1]);
}

// (R, E, literal-path entries, fine cells, thin entries, sort-path entries) of a binning (dgs_binning_info).
extern "C" int dgs_test_radix_sort(int64_t n, int bits, int key_bytes, const void *kin, void *kout,
                                   const uint32_t *vin, uint32_t *vout, dgs_stream_t stream);

// The binning's radix sort on its own (tests/test_gpu_radix.py): keys int16 / int32 (bit
// patterns), values int32; returns the stably sorted pair.
std::tuple<Tensor, Tensor> RadixSortTest(const Tensor &keys_in, const Tensor &vals_in, int64_t bits) {
    TORCH_CHECK(keys_in.is_cuda() && vals_in.is_cuda(), "radix_sort_test: CUDA tensors");
    TORCH_CHECK(keys_in.scalar_type() == at::kShort || keys_in.scalar_type() == at::kInt, "keys int16 / int32");
    TORCH_CHECK(vals_in.scalar_type() == at::kInt && vals_in.numel() == keys_in.numel(), "values int32, same length");
    const Tensor keys = keys_in.contiguous(), vals = vals_in.contiguous();
    Tensor ko = torch::empty_like(keys), vo = torch::empty_like(vals);
    check(dgs_test_radix_sort(keys.numel(), (int)bits, (int)keys.element_size(), keys.data_ptr(), ko.data_ptr(),
                              reinterpret_cast<const uint32_t *>(vals.data_ptr<int32_t>()),
                              reinterpret_cast<uint32_t *>(vo.data_ptr<int32_t>()), as_dgs(cur_stream())),
          "radix_sort_test");
    return std::make_tuple(ko, vo);
}

extern "C" int dgs_debug_fc_prof(unsigned long long *out8);
std::vector<int64_t> DebugFcProf() {
    unsigned long long o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    check(dgs_debug_fc_prof(o), "debug_fc_prof");
    return std::vector<int64_t>(o, o + 8);
}

std::tuple<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t> BinningInfo(const Tensor &binning_in,
                                                                               const Tensor &sbinning_in) {
    const Tensor gb = u8(binning_in, "binning_buffer"), sb = u8(sbinning_in, "sample_binning_buffer");
    int64_t o[6] = {0, 0, 0, 0, 0, 0};
    check(dgs_binning_info(gb.data_ptr(), (size_t)gb.numel(), sb.data_ptr(), (size_t)sb.numel(), o), "binning_info");
    return std::make_tuple(o[0], o[1], o[2], o[3], o[4], o[5]);
}

// Whether forward / backward with these tensors take the binned path (dgs_inputs_match).
bool InputsMatch(const Tensor &means_in, const Tensor &conics_in, const Tensor &samples_in,
                 const Tensor &binning_in, const Tensor &sbinning_in) {
    const Tensor means = f32(means_in, "means"), conics = f32(conics_in, "conics");
    const Tensor samples = f32(samples_in, "samples");
    const int P = (int)means.size(0), D = (int)means.size(-1), N = (int)samples.size(0);
    int match = 1;
    if (P != 0 && N != 0) {
        const Tensor gb = u8(binning_in, "binning_buffer"), sb = u8(sbinning_in, "sample_binning_buffer");
        check(dgs_inputs_match(P, D, N, means.data_ptr<float>(), conics.data_ptr<float>(), samples.data_ptr<float>(),
                               gb.data_ptr(), (size_t)gb.numel(), sb.data_ptr(), (size_t)sb.numel(), &match,
                               as_dgs(cur_stream())),
              "inputs_match");
    }
    return match != 0;
}

// The C-ABI tile grid (device min/max, torch-CUDA arithmetic) -- for tests of dgs_tile_grid.
// SupportExchange's sets (distributed.py): (mask int32 [P] bit per rank, owner int32 [P]).
std::tuple<Tensor, Tensor> ExchangeSets(const Tensor &means_in, const Tensor &conics_in,
                                        const std::vector<double> &extents) {
    const Tensor means = f32(means_in, "means"), conics = f32(conics_in, "conics");
    const int P = (int)means.size(0), D = (int)means.size(-1);
    const int W = (int)(extents.size() / 2);
    Tensor mask = torch::empty({P}, means.options().dtype(torch::kInt32));
    Tensor owner = torch::empty({P}, means.options().dtype(torch::kInt32));
    check(dgs_exchange_sets(P, D, means.data_ptr<float>(), conics.data_ptr<float>(), W, extents.data(),
                            reinterpret_cast<uint32_t *>(mask.data_ptr<int>()), owner.data_ptr<int>(),
                            as_dgs(cur_stream())),
          "exchange_sets");
    return std::make_tuple(mask, owner);
}

std::tuple<std::vector<int>, std::vector<float>> TileGrid(const Tensor &samples_in) {
    const Tensor samples = f32(samples_in, "samples");
    const int N = (int)samples.size(0), D = (int)samples.size(-1);
    std::vector<int> grid(D);
    std::vector<float> off(D);
    check(dgs_tile_grid(N, D, samples.data_ptr<float>(), grid.data(), off.data(), as_dgs(cur_stream())),
          "tile_grid");
    return std::make_tuple(grid, off);
}

// ---- neighbour aggregation (aggregate_neighbors.h:11-47) --------------------------------

// Per preprocess_aggregate call: the spatial row order (a scheduling hint: any permutation of
// 0..P-1 gives identical results, so a stale entry whose key was reused by another tensor of the
// same P costs speed at most) and the transposed lists of dgs_agg_transpose (results depend on
// them: used only while the very indices tensor they were built from is alive and unmodified --
// a weak reference to it and its version counter).
struct AggEntry {
    const void *indices;
    int64_t P, length;
    Tensor order;
    WeakImpl impl;
    int64_t version;
    Tensor tstart, tslot, rstart;  // undefined: not built
    Tensor ranges;                 // (the record layout follows the row lengths too)
    int64_t ranges_version;
};
std::mutex g_agg_mu;
std::vector<AggEntry> g_agg;

void agg_put(const Tensor &indices, const Tensor &ranges, int64_t P, const Tensor &order, const Tensor &tstart,
             const Tensor &tslot, const Tensor &rstart) {
    std::lock_guard<std::mutex> lk(g_agg_mu);
    for (auto it = g_agg.begin(); it != g_agg.end();)
        if (it->indices == indices.data_ptr() || it->impl.expired()) it = g_agg.erase(it);
        else ++it;
    // (inference tensors have no version counter: their entry only carries the row order, a
    // scheduling hint, and never transposed lists: transpose_get / transpose_put skip them)
    const bool tr = trackable({&indices, &ranges});
    g_agg.push_back({indices.data_ptr(), P, indices.numel(), order, WeakImpl(indices.getIntrusivePtr()),
                     tr ? (int64_t)indices._version() : -1, tr ? tstart : Tensor(), tr ? tslot : Tensor(),
                     tr ? rstart : Tensor(), ranges, tr ? (int64_t)ranges._version() : -1});
    if (g_agg.size() > 2) g_agg.erase(g_agg.begin());
}

const int32_t *order_get(const Tensor &indices, int64_t P) {
    std::lock_guard<std::mutex> lk(g_agg_mu);
    for (const auto &e : g_agg)
        if (e.indices == indices.data_ptr() && e.P == P && e.length == indices.numel() &&
            e.order.device() == indices.device())
            return e.order.data_ptr<int32_t>();
    return nullptr;
}

// The transposed lists built from exactly this indices tensor (same object, not modified since).
// Entries whose indices tensor has died are dropped here too (they would pin their lists).
bool transpose_get(const Tensor &indices, const Tensor &ranges, int64_t P, Tensor &tstart, Tensor &tslot,
                   Tensor &rstart) {
    if (!trackable({&indices, &ranges})) return false;
    std::lock_guard<std::mutex> lk(g_agg_mu);
    for (auto it = g_agg.begin(); it != g_agg.end();)
        if (it->impl.expired()) it = g_agg.erase(it);
        else ++it;
    for (const auto &e : g_agg) {
        if (!e.tstart.defined() || e.P != P || e.length != indices.numel()) continue;
        const auto sp = e.impl.lock();
        if (sp.get() == indices.unsafeGetTensorImpl() && e.version == (int64_t)indices._version() &&
            e.ranges.data_ptr() == ranges.data_ptr() && e.ranges_version == (int64_t)ranges._version()) {
            tstart = e.tstart;
            tslot = e.tslot;
            rstart = e.rstart;
            return true;
        }
    }
    return false;
}

// Keeps lists built at a backward call with the cache entry of the indices tensor they came from
// (built lazily: forward-only users never pay for the transposition).
void transpose_put(const Tensor &indices, const Tensor &ranges, int64_t P, const Tensor &tstart, const Tensor &tslot,
                   const Tensor &rstart) {
    if (!trackable({&indices, &ranges})) return;
    std::lock_guard<std::mutex> lk(g_agg_mu);
    for (auto &e : g_agg) {
        if (e.P != P || e.length != indices.numel()) continue;
        const auto sp = e.impl.lock();
        if (sp.get() == indices.unsafeGetTensorImpl() && e.version == (int64_t)indices._version() &&
            e.ranges.data_ptr() == ranges.data_ptr() && e.ranges_version == (int64_t)ranges._version()) {
            e.tstart = tstart;
            e.tslot = tslot;
            e.rstart = rstart;
            return;
        }
    }
}

bool transpose_enabled() {
    const char *e = std::getenv("DGS_AGG_TRANSPOSE");
    return !(e && e[0] == '0');
}

// dgs_agg_transpose into fresh tensors.
void build_transpose(const Tensor &indices, const Tensor &ranges, const int32_t *order, int64_t P, Tensor &tstart,
                     Tensor &tslot, Tensor &rstart, bool debug) {
    const int64_t length = indices.numel();
    tstart = torch::empty({P + 1}, indices.options().dtype(torch::kInt32));
    tslot = torch::empty({std::max<int64_t>(length, 1)}, indices.options().dtype(torch::kInt32));
    rstart = torch::empty({std::max<int64_t>(P, 1)}, indices.options().dtype(torch::kInt32));
    AllocCtx ctx{indices.device()};
    check(dgs_agg_transpose((int)P, length, indices.data_ptr<int64_t>(), ranges.data_ptr<int64_t>(), order,
                            tstart.data_ptr<int32_t>(), reinterpret_cast<uint32_t *>(tslot.data_ptr<int32_t>()),
                            rstart.data_ptr<int32_t>(), alloc_cb, &ctx, as_dgs(cur_stream()), debug ? 1 : 0),
          "preprocess_aggregate (transpose)");
}

Tensor i64(const Tensor &t, const char *name) {
    TORCH_CHECK(t.scalar_type() == torch::kInt64, name, " must be an int64 tensor (got ", t.scalar_type(), ")");
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    return t.contiguous();
}

// AggregateNeighborsPreprocessCUDA (aggregate_neighbors.cu:323-367)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> AggregateNeighborsPreprocessCUDA(
    const Tensor &means_in, const Tensor &conics_in, const Tensor &radii_in, const bool debug) {
    const Tensor means = f32(means_in, "means"), conics = f32(conics_in, "conics");
    const Tensor radii = f32(radii_in, "radii");
    const int P = (int)means.size(0), D = (int)means.size(-1);
    const auto lopt = means.options().dtype(torch::kInt64);
    Tensor ranges = torch::zeros({P}, lopt);
    Tensor inv_total = torch::zeros({P}, means.options());
    AllocCtx ctx{means.device()};
    int64_t length = 0;
    Tensor order = torch::empty({P}, means.options().dtype(torch::kInt32));
    if (P != 0) {
        TORCH_CHECK(D == 1 || D == 2, "only D = 1 or D = 2 is supported");
        TORCH_CHECK(radii.numel() == P && conics.size(0) == P, "means, conics and radii must have P rows");
        check(dgs_agg_preprocess(P, D, means.data_ptr<float>(), conics.data_ptr<float>(), radii.data_ptr<float>(),
                                 ranges.data_ptr<int64_t>(), inv_total.data_ptr<float>(), order.data_ptr<int32_t>(),
                                 alloc_cb, &ctx, &length,
                                 as_dgs(cur_stream()), debug ? 1 : 0),
              "preprocess_aggregate");
    }
    auto view = [&](int which, torch::ScalarType st, std::vector<int64_t> shape) {
        if (length == 0) return torch::empty(shape, means.options().dtype(st));
        return ctx.bufs[which].view(st).narrow(0, 0, length * (shape.size() > 1 ? shape[1] : 1)).view(shape);
    };
    Tensor indices = view(DGS_BUF_AGG_INDICES, torch::kInt64, {length});
    // (the transposed lists of the backward's per-row gather, dgs_agg_backward_tr, are built at
    // the first backward on these lists and kept with this entry)
    if (length > 0) agg_put(indices, ranges, P, order, Tensor(), Tensor(), Tensor());
    return std::make_tuple(indices, ranges, view(DGS_BUF_AGG_DISTS, torch::kFloat32, {length, D}),
                           view(DGS_BUF_AGG_DENSITIES, torch::kFloat32, {length}), inv_total);
}

struct AggIn {
    Tensor features, transform, queries, keys, freq, dt, indices, ranges, dists, densities, inv_total;
    int P, D, L, K, E;
};

AggIn agg_inputs(const Tensor &features, const Tensor &transform, const Tensor &queries, const Tensor &keys,
                 const Tensor &frequencies, const Tensor &distance_transform, const Tensor &indices,
                 const Tensor &ranges, const Tensor &dists, const Tensor &densities, const Tensor &inv_total) {
    AggIn a;
    a.features = f32(features, "features"), a.transform = f32(transform, "transform");
    a.queries = f32(queries, "queries"), a.keys = f32(keys, "keys");
    a.freq = f32(frequencies, "frequencies"), a.dt = f32(distance_transform, "distance_transform");
    a.indices = i64(indices, "indices"), a.ranges = i64(ranges, "ranges");
    a.dists = f32(dists, "dists"), a.densities = f32(densities, "densities");
    a.inv_total = f32(inv_total, "inv_total_densities");
    // aggregate_neighbors.cu:383-387
    a.P = (int)a.features.size(0), a.D = (int)a.dists.size(-1), a.L = (int)a.features.size(-1);
    a.K = (int)a.queries.size(-1), a.E = (int)(a.dt.size(-1) / 2);
    TORCH_CHECK(a.ranges.numel() == a.P && a.inv_total.numel() == a.P, "ranges / inv_total must have P entries");
    TORCH_CHECK(a.transform.numel() == (int64_t)a.L * a.L, "transform must be L x L");
    TORCH_CHECK(a.keys.numel() == (int64_t)a.P * a.K && a.queries.numel() == (int64_t)a.P * a.K,
                "queries / keys must be P x K");
    const int F = a.E >= 1 ? (a.E - 1) / a.D / 2 : 0;
    TORCH_CHECK(a.freq.numel() >= F, "frequencies must hold (E-1)/D/2 entries");
    TORCH_CHECK(a.indices.numel() == a.densities.numel() && a.dists.numel() == a.indices.numel() * a.D,
                "indices / dists / densities must come from preprocess_aggregate");
    return a;
}

// AggregateNeighborsCUDA (aggregate_neighbors.cu:369-415)
std::tuple<Tensor, Tensor, Tensor, Tensor> AggregateNeighborsCUDA(
    const Tensor &features, const Tensor &transform, const Tensor &queries, const Tensor &keys,
    const Tensor &frequencies, const Tensor &distance_transform, const Tensor &indices, const Tensor &ranges,
    const Tensor &dists, const Tensor &densities, const Tensor &inv_total_densities, const bool debug) {
    const AggIn a = agg_inputs(features, transform, queries, keys, frequencies, distance_transform, indices,
                               ranges, dists, densities, inv_total_densities);
    Tensor weights = torch::zeros(a.densities.sizes(), a.features.options());
    Tensor embeddings = torch::zeros(a.densities.sizes(), a.features.options());
    Tensor factors = torch::zeros(a.densities.sizes(), a.features.options());
    Tensor out = torch::zeros({a.P, a.L}, a.features.options());
    check(dgs_agg_forward(a.P, a.D, a.L, a.K, a.E, a.features.data_ptr<float>(), a.transform.data_ptr<float>(),
                          a.queries.data_ptr<float>(), a.keys.data_ptr<float>(), a.freq.data_ptr<float>(),
                          a.dt.data_ptr<float>(), a.indices.data_ptr<int64_t>(), a.ranges.data_ptr<int64_t>(),
                          a.dists.data_ptr<float>(), a.densities.data_ptr<float>(), a.inv_total.data_ptr<float>(),
                          order_get(a.indices, a.P), weights.data_ptr<float>(), embeddings.data_ptr<float>(), factors.data_ptr<float>(),
                          out.data_ptr<float>(), as_dgs(cur_stream()), debug ? 1 : 0),
          "aggregate_neighbors");
    return std::make_tuple(weights, embeddings, factors, out);
}

// AggregateNeighborsBackwardCUDA (aggregate_neighbors.cu:417-475)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> AggregateNeighborsBackwardCUDA(
    const Tensor &features, const Tensor &transform, const Tensor &queries, const Tensor &keys,
    const Tensor &frequencies, const Tensor &distance_transform, const Tensor &indices, const Tensor &ranges,
    const Tensor &dists, const Tensor &densities, const Tensor &weights_in, const Tensor &embeddings_in,
    const Tensor &factors_in, const Tensor &inv_total_densities, const Tensor &dL_in, const bool debug) {
    const AggIn a = agg_inputs(features, transform, queries, keys, frequencies, distance_transform, indices,
                               ranges, dists, densities, inv_total_densities);
    const Tensor weights = f32(weights_in, "weights"), embeddings = f32(embeddings_in, "embeddings");
    const Tensor factors = f32(factors_in, "factors"), dL = f32(dL_in, "dL_dneighbor_features");
    TORCH_CHECK(dL.numel() == (int64_t)a.P * a.L, "dL_dneighbor_features must be P x L");
    Tensor dfeat = torch::zeros(a.features.sizes(), a.features.options());
    Tensor dtrans = torch::zeros(a.transform.sizes(), a.features.options());
    Tensor dq = torch::zeros(a.queries.sizes(), a.features.options());
    Tensor dkeys = torch::zeros(a.keys.sizes(), a.features.options());
    Tensor dfreq = torch::zeros(a.freq.sizes(), a.features.options());
    Tensor ddt = torch::zeros(a.dt.sizes(), a.features.options());
    const int64_t length = a.indices.numel();
    Tensor tstart, tslot, rstart;
    const bool tr = a.P > 0 && a.L + a.K <= 64 && length < ((int64_t)1 << 31) && transpose_enabled();
    if (tr && !transpose_get(a.indices, a.ranges, a.P, tstart, tslot, rstart)) {  // first backward on these lists
        build_transpose(a.indices, a.ranges, order_get(a.indices, a.P), a.P, tstart, tslot, rstart, debug);
        transpose_put(a.indices, a.ranges, a.P, tstart, tslot, rstart);
    }
    if (tr) {
        const size_t ws = dgs_agg_workspace_size_tr(a.P, a.L, length);
        Tensor work = torch::empty({(int64_t)ws}, a.features.options().dtype(torch::kUInt8));
        check(dgs_agg_backward_tr(a.P, a.D, a.L, a.K, a.E, a.features.data_ptr<float>(), a.transform.data_ptr<float>(),
                                  a.queries.data_ptr<float>(), a.keys.data_ptr<float>(), a.freq.data_ptr<float>(),
                                  a.dt.data_ptr<float>(), a.indices.data_ptr<int64_t>(), a.ranges.data_ptr<int64_t>(),
                                  a.dists.data_ptr<float>(), a.densities.data_ptr<float>(), weights.data_ptr<float>(),
                                  embeddings.data_ptr<float>(), factors.data_ptr<float>(), a.inv_total.data_ptr<float>(),
                                  order_get(a.indices, a.P), tstart.data_ptr<int32_t>(),
                                  reinterpret_cast<const uint32_t *>(tslot.data_ptr<int32_t>()),
                                  rstart.data_ptr<int32_t>(), length,
                                  dL.data_ptr<float>(), dfeat.data_ptr<float>(), dtrans.data_ptr<float>(),
                                  dq.data_ptr<float>(), dkeys.data_ptr<float>(), dfreq.data_ptr<float>(),
                                  ddt.data_ptr<float>(), work.data_ptr(), ws, as_dgs(cur_stream()), debug ? 1 : 0),
              "aggregate_neighbors_backward");
        return std::make_tuple(dfeat, dtrans, dq, dkeys, dfreq, ddt);
    }
    const size_t ws = dgs_agg_workspace_size(a.P, a.L);
    Tensor work = torch::empty({(int64_t)ws}, a.features.options().dtype(torch::kUInt8));
    check(dgs_agg_backward(a.P, a.D, a.L, a.K, a.E, a.features.data_ptr<float>(), a.transform.data_ptr<float>(),
                           a.queries.data_ptr<float>(), a.keys.data_ptr<float>(), a.freq.data_ptr<float>(),
                           a.dt.data_ptr<float>(), a.indices.data_ptr<int64_t>(), a.ranges.data_ptr<int64_t>(),
                           a.dists.data_ptr<float>(), a.densities.data_ptr<float>(), weights.data_ptr<float>(),
                           embeddings.data_ptr<float>(), factors.data_ptr<float>(), a.inv_total.data_ptr<float>(),
                           order_get(a.indices, a.P), dL.data_ptr<float>(), dfeat.data_ptr<float>(), dtrans.data_ptr<float>(),
                           dq.data_ptr<float>(), dkeys.data_ptr<float>(), dfreq.data_ptr<float>(),
                           ddt.data_ptr<float>(), work.data_ptr(), ws, as_dgs(cur_stream()), debug ? 1 : 0),
          "aggregate_neighbors_backward");
    return std::make_tuple(dfeat, dtrans, dq, dkeys, dfreq, ddt);
}

// ---- D = 3 fields (include/dgs_volume.h; beyond the reference) --------
void vol_shapes(const Tensor &means, const Tensor &conics, const Tensor &samples) {
    TORCH_CHECK(means.dim() == 2 && means.size(1) == 3, "volume: means must be [P, 3]");
    TORCH_CHECK(conics.dim() == 2 && conics.size(1) == 6 && conics.size(0) == means.size(0),
                "volume: conics must be [P, 6] (packed c00 c01 c02 c11 c12 c22)");
    TORCH_CHECK(samples.dim() == 2 && samples.size(1) == 3, "volume: samples must be [N, 3]");
}

Tensor VolumePreprocess(const Tensor &means_in, const Tensor &conics_in, const Tensor &samples_in,
                        const bool debug) {
    const Tensor means = f32(means_in, "means"), conics = f32(conics_in, "conics");
    const Tensor samples = f32(samples_in, "samples");
    vol_shapes(means, conics, samples);
    AllocCtx ctx{means.device(), {}, {}};
    check(dgs_volume_preprocess((int)means.size(0), (int)samples.size(0), means.data_ptr<float>(),
                                conics.data_ptr<float>(), samples.data_ptr<float>(), alloc_cb, &ctx,
                                as_dgs(cur_stream()), debug ? 1 : 0),
          "volume_preprocess");
    return ctx.bufs[DGS_BUF_BINNING];
}

Tensor VolumeForward(int function, const Tensor &means_in, const Tensor &values_in, const Tensor &conics_in,
                     const Tensor &samples_in, const Tensor &binning_in, const bool debug) {
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    const Tensor conics = f32(conics_in, "conics"), samples = f32(samples_in, "samples");
    const Tensor binning = u8(binning_in, "binning_buffer");
    vol_shapes(means, conics, samples);
    TORCH_CHECK(function >= 0 && function <= 3, "volume: function must be 0..3");
    TORCH_CHECK(values.dim() == 2 && values.size(0) == means.size(0), "volume: values must be [P, C]");
    const int64_t P = means.size(0), N = samples.size(0), C = values.size(1);
    std::vector<int64_t> shape{N};
    for (int k = 0; k < function; ++k) shape.push_back(3);
    shape.push_back(C);
    Tensor out = torch::zeros(shape, means.options());
    if (N == 0 || C == 0) return out;
    check(dgs_volume_forward(function, (int)P, (int)N, (int)C, means.data_ptr<float>(), values.data_ptr<float>(),
                             conics.data_ptr<float>(), samples.data_ptr<float>(), binning.data_ptr(),
                             (size_t)binning.numel(), out.data_ptr<float>(), as_dgs(cur_stream()), debug ? 1 : 0),
          "volume_forward");
    return out;
}

std::tuple<Tensor, Tensor, Tensor> VolumeBackward(int function, const Tensor &means_in, const Tensor &values_in,
                                                  const Tensor &conics_in, const Tensor &samples_in,
                                                  const Tensor &binning_in, const Tensor &dL_in, const bool debug) {
    const Tensor means = f32(means_in, "means"), values = f32(values_in, "values");
    const Tensor conics = f32(conics_in, "conics"), samples = f32(samples_in, "samples");
    const Tensor binning = u8(binning_in, "binning_buffer"), dL = f32(dL_in, "dL_dout");
    vol_shapes(means, conics, samples);
    TORCH_CHECK(function >= 0 && function <= 3, "volume: function must be 0..3");
    const int64_t P = means.size(0), N = samples.size(0), C = values.size(1);
    int64_t K = 1;
    for (int k = 0; k < function; ++k) K *= 3;
    TORCH_CHECK(dL.numel() == N * K * C, "volume: dL_dout must be [N, 3^function, C]");
    Tensor dm = torch::zeros({P, 3}, means.options()), dv = torch::zeros({P, C}, means.options());
    Tensor dc = torch::zeros({P, 6}, means.options());
    if (P == 0 || C == 0) return std::make_tuple(dm, dv, dc);
    const size_t ws = dgs_volume_workspace_size(function, (int)P, (int)N, (int)C, 1);
    Tensor work = torch::empty({(int64_t)std::max<size_t>(ws, 4)}, means.options().dtype(torch::kUInt8));
    check(dgs_volume_backward(function, (int)P, (int)N, (int)C, means.data_ptr<float>(), values.data_ptr<float>(),
                              conics.data_ptr<float>(), samples.data_ptr<float>(), dL.data_ptr<float>(),
                              binning.data_ptr(), (size_t)binning.numel(), dm.data_ptr<float>(),
                              dv.data_ptr<float>(), dc.data_ptr<float>(), work.data_ptr(), ws,
                              as_dgs(cur_stream()), debug ? 1 : 0),
          "volume_backward");
    return std::make_tuple(dm, dv, dc);
}

std::tuple<int64_t, int64_t> VolumeCountPairs(const Tensor &means_in, const Tensor &conics_in,
                                              const Tensor &samples_in, const Tensor &binning_in) {
    const Tensor means = f32(means_in, "means"), conics = f32(conics_in, "conics");
    const Tensor samples = f32(samples_in, "samples"), binning = u8(binning_in, "binning_buffer");
    vol_shapes(means, conics, samples);
    int64_t c[2] = {0, 0};
    check(dgs_volume_count_pairs((int)means.size(0), (int)samples.size(0), means.data_ptr<float>(),
                                 conics.data_ptr<float>(), samples.data_ptr<float>(), binning.data_ptr(),
                                 (size_t)binning.numel(), c, as_dgs(cur_stream())),
          "volume_count_pairs");
    return std::make_tuple(c[0], c[1]);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.doc() = "MI355X-native differentiable Gaussian sampling (HIP / gfx950)";
    // ext.cpp:20-31
    m.def("preprocess_gaussians", &PreprocessCUDA);
    m.def("sample_gaussians", &SampleGaussiansCUDA);
    m.def("sample_gaussians_backward", &SampleGaussiansBackwardCUDA);
    m.def("sample_gaussians_derivative", &SampleGaussiansDerivativeCUDA);
    m.def("sample_gaussians_derivative_backward", &SampleGaussiansDerivativeBackwardCUDA);
    m.def("sample_gaussians_laplacian", &SampleGaussiansLaplacianCUDA);
    m.def("sample_gaussians_laplacian_backward", &SampleGaussiansLaplacianBackwardCUDA);
    m.def("sample_gaussians_third_derivative", &SampleGaussiansThirdCUDA);
    m.def("sample_gaussians_third_derivative_backward", &SampleGaussiansThirdBackwardCUDA);
    m.def("aggregate_neighbors", &AggregateNeighborsCUDA);
    m.def("aggregate_neighbors_backward", &AggregateNeighborsBackwardCUDA);
    m.def("preprocess_aggregate", &AggregateNeighborsPreprocessCUDA);
    // extensions (not on the reference surface)
    m.def("preprocess_gaussians_bounded", &PreprocessBoundedCUDA);
    m.def("preprocess_gaussians_sharded", &PreprocessShardedCUDA);
    m.def("count_pairs", &CountPairs);
    m.def("sample_gaussians_multi", &SampleGaussiansMulti);
    m.def("sample_gaussians_multi_backward", &SampleGaussiansMultiBackward);
    m.def("tile_grid", &TileGrid);
    m.def("exchange_sets", &ExchangeSets);
    m.def("inputs_match", &InputsMatch);
    m.def("binning_info", &BinningInfo);
    m.def("preprocess_gaussians_capturable", &PreprocessCapturableCUDA);
    m.def("radix_sort_test", &RadixSortTest);
    m.def("debug_fc_prof", &DebugFcProf);
    m.def("volume_preprocess", &VolumePreprocess);
    m.def("volume_forward", &VolumeForward);
    m.def("volume_backward", &VolumeBackward);
    m.def("volume_count_pairs", &VolumeCountPairs);
    m.def("library_version", []() { return dgs_version(); });
    m.def("warmup", []() { check(dgs_warmup(as_dgs(cur_stream())), "warmup"); });
    m.def("timing_enable", [](bool on) { dgs_timing_enable(on ? 1 : 0); });
    m.def("timing_read", [](int which) {
        double ms = 0.0;
        const int n = dgs_timing_read(which, &ms);
        return std::make_tuple(n, ms);
    });
}
