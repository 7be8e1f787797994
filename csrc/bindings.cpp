// Python bindings of the gfx950 kernels (torch extension module `pytorch_distributed_template_amd._C`).
//
// The binding layer is deliberately thin: it validates tensors (device, dtype, contiguity, sizes
// that the kernels' grids assume) and forwards raw pointers plus the current PyTorch HIP stream to
// the launchers in csrc/kernels/*.hip.  Every kernel is enqueued on the caller's current stream, so
// the ops compose with PyTorch's stream semantics, hipGraph capture and RCCL's stream ordering.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>

#include <cstdio>
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <vector>
#include <stdexcept>
#include <string>

#include "dtypes.h"
#include "kernels/bn.h"
#include "kernels/conv1x1.h"
#include "kernels/conv_fwd.h"
#include "kernels/conv_l1.h"
#include "kernels/conv_wgrad.h"
#include "kernels/fp32.h"
#include "kernels/loss.h"
#include "kernels/optim.h"
#include "kernels/pool.h"
#include "kernels/stem.h"
#include "kernels/vgg.h"

namespace pdt_comm {
void register_comm(pybind11::module& m);  // csrc/comm.cpp
}
namespace pdt_store {
void register_store(pybind11::module& m);  // csrc/store.cpp
}
namespace pdt_dp {
void register_dp(pybind11::module& m);  // csrc/dp_group.cpp
}

void pdt_hip_fail(const char* expr, hipError_t e, const char* file, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), "%s failed: %s (%s:%d)", expr, hipGetErrorString(e), file, line);
  throw std::runtime_error(buf);
}

// ------------------------------------------------------------------------------- dispatch counters
namespace pdt {
namespace {
struct CounterRegistry {
  std::mutex mu;
  std::vector<std::pair<std::string, std::unique_ptr<long long>>> entries;
};
CounterRegistry& counters() {
  static CounterRegistry r;
  return r;
}
}  // namespace
long long* dispatch_counter(const char* name) {
  auto& r = counters();
  std::lock_guard<std::mutex> lk(r.mu);
  for (auto& e : r.entries)
    if (e.first == name) return e.second.get();
  r.entries.emplace_back(name, std::make_unique<long long>(0));
  return r.entries.back().second.get();
}

void* scratch_alloc(size_t bytes, hipStream_t s) {
  void* p = c10::hip::HIPCachingAllocator::raw_alloc_with_stream(bytes, s);
  // PDT_SCRATCH_POISON=1 (debugging): fill every internal scratch buffer with 0xFF bytes (NaN) before the kernels
  // that are meant to write all of it -- any element they leave unwritten then surfaces as NaN downstream
  static const bool poison = [] {
    const char* e = getenv("PDT_SCRATCH_POISON");
    return e && e[0] == '1';
  }();
  if (poison && p && bytes) {
    hipError_t e = hipMemsetAsync(p, 0xFF, bytes, s);
    if (e != hipSuccess) pdt_hip_fail("hipMemsetAsync(scratch poison)", e, __FILE__, __LINE__);
  }
  return p;
}
void scratch_free(void* p) { c10::hip::HIPCachingAllocator::raw_delete(p); }
}  // namespace pdt

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// after every kernel launch of a binding: a launch the runtime refused (LDS / register / grid limits) raises here
// instead of leaving its output buffer stale
void launched(const char* op) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, op, ": kernel launch failed: ", hipGetErrorString(e));
}

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, ": expected a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, ": expected a contiguous tensor");
}

int dt16(const Tensor& t, const char* name) {
  check_dev(t, name);
  if (t.scalar_type() == at::kBFloat16) return pdt::kBF16;
  if (t.scalar_type() == at::kHalf) return pdt::kF16;
  TORCH_CHECK(false, name, ": expected bfloat16 or float16, got ", t.scalar_type());
}

uint16_t* p16(const Tensor& t, const char* name) {
  dt16(t, name);
  return reinterpret_cast<uint16_t*>(t.data_ptr());
}
const uint16_t* p16o(const OptT& t, const char* name) { return t.has_value() ? p16(*t, name) : nullptr; }
uint16_t* p16m(const OptT& t, const char* name) { return t.has_value() ? p16(*t, name) : nullptr; }

float* pf(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, ": expected float32");
  return t.data_ptr<float>();
}
float* pfo(const OptT& t, const char* name) { return t.has_value() ? pf(*t, name) : nullptr; }

// ReLU bitmask (bit e of byte v = element 8v+e > 0) of a 16-bit activation with `n` elements
uint8_t* pmask(const OptT& t, int64_t n, const char* name) {
  if (!t.has_value()) return nullptr;
  check_dev(*t, name);
  TORCH_CHECK(t->scalar_type() == at::kByte, name, ": expected a uint8 bitmask");
  TORCH_CHECK(n % 8 == 0 && t->numel() == n / 8, name, ": bitmask must hold numel/8 bytes");
  return t->data_ptr<uint8_t>();
}

double* pd(const Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kDouble, name, ": expected float64");
  return t.data_ptr<double>();
}

// ------------------------------------------------------------------------------------------ conv
void conv_fwd(const Tensor& x, const Tensor& w, Tensor& y, const OptT& res, const OptT& stats, int64_t N, int64_t H,
              int64_t W, int64_t C, int64_t Kout, int64_t T, int64_t U, int64_t Pm, int64_t Qm, int64_t ist_h,
              int64_t ist_w, int64_t ioff_h, int64_t ioff_w, int64_t tstep_h, int64_t tstep_w, int64_t OH, int64_t OW,
              int64_t ost_h, int64_t ost_w, int64_t ooff_h, int64_t ooff_w, int64_t bm, int64_t bn, int64_t bk,
              int64_t cs) {
  const int dt = dt16(x, "x");
  if (cs <= 0) cs = C;
  TORCH_CHECK(dt16(w, "w") == dt && dt16(y, "y") == dt, "conv_fwd: mixed dtypes");
  TORCH_CHECK(x.numel() == N * H * W * cs, "conv_fwd: x has ", x.numel(), " elements, geometry needs ", N * H * W * cs);
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && w.numel() < (int64_t(1) << 30),
              "conv_fwd: operands exceed 2 GiB (32-bit buffer offsets)");
  int pair_skip = 0;
  if (cs != C) {  // window mode: every tap's C-element chunk must stay inside the padded image
    // C == 32: one kernel row per tap; C == 64: two consecutive kernel rows per tap (BK must be 64)
    const int rows = C == 64 ? 2 : 1;
    // U > 1 column taps (C == 32 only): windows tstep_w pixels apart, e.g. AlexNet's 11-wide kernel rows as two
    // 8-pixel windows
    TORCH_CHECK(cs == 4 && (C == 32 || (C == 64 && bk == 64 && U == 1)) && tstep_w >= 0 && U >= 1 && ioff_h >= 0 &&
                    ioff_w >= 0 && (Pm - 1) * ist_h + ioff_h + (T - 1) * tstep_h + rows - 1 < H &&
                    ((Qm - 1) * ist_w + ioff_w + (U - 1) * tstep_w) * cs + 32 <= W * cs,
                "conv_fwd: window-mode geometry leaves the padded image");
    if (C == 64) pair_skip = (int)(W * cs - 32);
  }
  TORCH_CHECK(w.numel() == Kout * T * U * C, "conv_fwd: w size mismatch");
  TORCH_CHECK(y.numel() == N * OH * OW * Kout, "conv_fwd: y size mismatch");
  TORCH_CHECK(C % bk == 0 && Kout % bn == 0, "conv_fwd: C % bk / Kout % bn must be 0 (C=", C, " Kout=", Kout, ")");
  TORCH_CHECK(ost_h >= 1 && ost_w >= 1 && (Pm - 1) * ost_h + ooff_h < OH && (Qm - 1) * ost_w + ooff_w < OW,
              "conv_fwd: output sub-grid exceeds the output tensor");
  pdt::ConvFwdArgs a{};
  a.x = p16(x, "x");
  a.w = p16(w, "w");
  a.y = p16(y, "y");
  if (res.has_value()) {
    TORCH_CHECK(res->numel() == y.numel(), "conv_fwd: residual size mismatch");
    a.res = p16(*res, "res");
  }
  const int64_t M = N * Pm * Qm;
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * Kout * 2, "conv_fwd: stats buffer too small");
    a.stats = pd(*stats, "stats");
  }
  a.N = N; a.H = H; a.W = W; a.C = C; a.Kout = Kout; a.T = T; a.U = U; a.Pm = Pm; a.Qm = Qm; a.cs = cs;
  a.pair_skip = pair_skip;
  a.ist_h = ist_h; a.ist_w = ist_w; a.ioff_h = ioff_h; a.ioff_w = ioff_w; a.tstep_h = tstep_h; a.tstep_w = tstep_w;
  a.OH = OH; a.OW = OW; a.ost_h = ost_h; a.ost_w = ost_w; a.ooff_h = ooff_h; a.ooff_w = ooff_w;
  TORCH_CHECK(M < (int64_t(1) << 31), "conv_fwd: N*Pm*Qm must be < 2^31 (32-bit pixel indexing)");
  a.M = M;
  pdt::conv_fwd_launch(a, dt, (int)bm, (int)bn, (int)bk, cur_stream());
  launched("conv_fwd_launch");
}

// ResNet layer1 3x3/s1/p1 64 -> 64 forward over the RAW output z of the block's first conv, with that conv's
// BatchNorm + ReLU (pre_coef = [scale(64) | shift(64) | ...]) applied inside the kernel to each staged input tile:
// y = conv(relu(bn(z))) with BN statistics of y, and relu(bn(z)) never written.
bool conv_fwd_pre_supported(int64_t N, int64_t H, int64_t W) {
  pdt::ConvFwdArgs a{};
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.C = 64; a.Kout = 64; a.T = 3; a.U = 3; a.cs = 64;
  a.Pm = (int)H; a.Qm = (int)W; a.ist_h = 1; a.ist_w = 1; a.ioff_h = -1; a.ioff_w = -1; a.tstep_h = 1;
  a.tstep_w = 1; a.OH = (int)H; a.OW = (int)W; a.ost_h = 1; a.ost_w = 1;
  int flip = 0;
  return pdt::conv_l1_eligible(a, &flip);
}

void conv_fwd_pre(const Tensor& z, const Tensor& w, Tensor& y, const Tensor& stats, const Tensor& pre_coef, int64_t N,
                  int64_t H, int64_t W) {
  const int dt = dt16(z, "z");
  TORCH_CHECK(dt16(w, "w") == dt && dt16(y, "y") == dt, "conv_fwd_pre: mixed dtypes");
  TORCH_CHECK(conv_fwd_pre_supported(N, H, W), "conv_fwd_pre: needs the layer1 geometry (64 -> 64, W == 56, H % 4 == 0)");
  TORCH_CHECK(z.numel() == N * H * W * 64 && y.numel() == z.numel() && w.numel() == 64 * 9 * 64,
              "conv_fwd_pre: size mismatch");
  TORCH_CHECK(z.numel() < (int64_t(1) << 30), "conv_fwd_pre: operands exceed 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(stats.numel() >= pdt::kStatSlots * 64 * 2, "conv_fwd_pre: stats buffer too small");
  TORCH_CHECK(pre_coef.numel() >= 128, "conv_fwd_pre: pre_coef needs scale[64] | shift[64]");
  pdt::ConvFwdArgs a{};
  a.x = p16(z, "z");
  a.w = p16(w, "w");
  a.y = p16(y, "y");
  a.stats = pd(stats, "stats");
  a.pre_coef = pf(pre_coef, "pre_coef");
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.C = 64; a.Kout = 64; a.T = 3; a.U = 3; a.cs = 64;
  a.Pm = (int)H; a.Qm = (int)W; a.ist_h = 1; a.ist_w = 1; a.ioff_h = -1; a.ioff_w = -1; a.tstep_h = 1;
  a.tstep_w = 1; a.OH = (int)H; a.OW = (int)W; a.ost_h = 1; a.ost_w = 1;
  a.M = N * H * W;
  pdt::conv_fwd_launch(a, dt, 256, 64, 64, cur_stream());
  launched("conv_fwd_launch");
}

// ResNet stem forward (7x7/2, 3 -> 64) over the zero-padded NHWC4 image with window-row weights
// [64][7][32]; optional fp64 BN statistics slots.
void stem_fwd(const Tensor& xp, const Tensor& w, Tensor& y, const OptT& stats, int64_t N, int64_t Hp, int64_t Wp,
              int64_t P, int64_t Q, int64_t blocks_per_cu) {
  const int dt = dt16(xp, "xp");
  TORCH_CHECK(dt16(w, "w") == dt && dt16(y, "y") == dt, "stem_fwd: mixed dtypes");
  TORCH_CHECK(xp.numel() == N * Hp * Wp * 4 && w.numel() == 64 * 7 * 32 && y.numel() == N * P * Q * 64,
              "stem_fwd: size mismatch");
  TORCH_CHECK(xp.numel() * 2 < (int64_t(1) << 31) && N * P * Q < (int64_t(1) << 31),
              "stem_fwd: input exceeds 2 GiB / 2^31 pixels (32-bit offsets)");
  TORCH_CHECK(pdt::stem_fwd_supported((int)Hp, (int)Wp, (int)P, (int)Q),
              "stem_fwd: unsupported geometry (needs Q <= 112, 13*Wp*8 <= 24 KiB and a padded image that covers "
              "every 7x7 window)");
  pdt::StemFwdArgs a{};
  a.x = p16(xp, "xp");
  a.x_bytes = (uint32_t)(xp.numel() * 2);
  a.w = p16(w, "w");
  a.y = p16(y, "y");
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * 64 * 2, "stem_fwd: stats buffer too small");
    a.stats = pd(*stats, "stats");
  }
  a.N = (int)N; a.Hp = (int)Hp; a.Wp = (int)Wp; a.P = (int)P; a.Q = (int)Q;
  a.blocks_per_cu = (int)std::max<int64_t>(1, blocks_per_cu);
  pdt::stem_fwd_launch(a, dt, cur_stream());
  launched("stem_fwd_launch");
}

int64_t conv_m_tiles(int64_t M, int64_t bm) { return pdt::conv_fwd_m_tiles(M, (int)bm); }

// Which persistent 1x1 backward-data kernel conv_dgrad_impl runs for a launch, if any: 0 none (tiled implicit GEMM),
// 1 conv1x1.hip (C = 256 -> K = 64 | 128), 2 conv1x1x.hip (sliced, layers 2-4).  The ONE source of this dispatch: the
// executor asks it (conv_dgrad_persistent) before choosing / autotuning a tile, so the two cannot drift apart.
static int dgrad_persistent_kind(int64_t K, int64_t C, int64_t bnb, int64_t stride,
                                 const std::vector<std::vector<int64_t>>& phases, int64_t H, int64_t W, int64_t P,
                                 int64_t Q, int64_t res_phase) {
  if (!(bnb == 2 || bnb == 3) || res_phase >= 0 || stride != 1 || phases.size() != 1 || H != P || W != Q) return 0;
  const auto& f = phases[0];
  if (f.size() < 6 || f[0] != 0 || f[1] != 0 || f[2] != 1 || f[3] != 1 || f[4] != 0 || f[5] != 0) return 0;
  const bool x_ok = pdt::conv1x1x_bnb_supported((int)K, (int)C);
  if ((K == 64 || (K == 128 && bnb == 2)) && C == 256 && pdt::conv1x1_c64_supported(64, C) &&
      !(pdt::conv1x1x_prefer_l1() && x_ok))
    return 1;
  return x_ok ? 2 : 0;
}

int64_t conv_dgrad_persistent(int64_t K, int64_t C, int64_t bnb, int64_t stride,
                              const std::vector<std::vector<int64_t>>& phases, int64_t H, int64_t W, int64_t P,
                              int64_t Q, int64_t res_phase) {
  return dgrad_persistent_kind(K, C, bnb, stride, phases, H, W, P, Q, res_phase);
}

// Backward-data of a (strided) conv in ONE launch: phases = [(ph, pw, T, U, ioff_h, ioff_w, woff), ...]
// over dY [N,P,Q,K] -> dX [N,H,W,C] (+ residual), wt = concatenated per-phase [C][T][U][K] weights.
void conv_dgrad_impl(const Tensor& dy, const Tensor& wt, Tensor& dx, const OptT& res, int64_t N, int64_t P,
                     int64_t Q, int64_t K, int64_t C, int64_t H, int64_t W, int64_t stride,
                     const std::vector<std::vector<int64_t>>& phases, int64_t bm, int64_t bn, int64_t bk, int64_t bnb,
                     const OptT& bn_y1, const OptT& bn_coef1, const OptT& bn_y2, const OptT& bn_coef2,
                     const OptT& bn_mask, const OptT& bn_slots, int64_t res_phase) {
  const int dt = dt16(dy, "dy");
  TORCH_CHECK(dt16(wt, "wt") == dt && dt16(dx, "dx") == dt, "conv_dgrad: mixed dtypes");
  TORCH_CHECK(dy.numel() == N * P * Q * K && dx.numel() == N * H * W * C, "conv_dgrad: size mismatch");
  TORCH_CHECK(dy.numel() < (int64_t(1) << 30) && wt.numel() < (int64_t(1) << 30),
              "conv_dgrad: operands exceed 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(!phases.empty() && phases.size() <= 4, "conv_dgrad: 1..4 phases");
  TORCH_CHECK(K % bk == 0 && C % bn == 0, "conv_dgrad: K % bk / C % bn must be 0");
  pdt::ConvFwdArgs a{};
  a.x = p16(dy, "dy");
  a.w = p16(wt, "wt");
  a.y = p16(dx, "dx");
  TORCH_CHECK(res_phase < (int64_t)phases.size() && (res_phase < 0 || res.has_value()), "conv_dgrad: bad res_phase");
  if (res.has_value()) {
    if (res_phase >= 0) {  // compact residual of one phase: [N * Pm * Qm][C] of that phase
      const auto& f = phases[res_phase];
      TORCH_CHECK(f.size() == 7, "conv_dgrad: phase = (ph, pw, T, U, ioff_h, ioff_w, woff)");
      const int64_t Pm = (H - f[0] + stride - 1) / stride, Qm = (W - f[1] + stride - 1) / stride;
      TORCH_CHECK(res->numel() == N * Pm * Qm * C, "conv_dgrad: compact residual size mismatch");
      // every phase reads the compact residual unconditionally (its add is selected per phase): its rows must
      // cover every phase's GEMM rows
      for (const auto& g : phases)
        TORCH_CHECK(g.size() == 7 && ((H - g[0] + stride - 1) / stride) * ((W - g[1] + stride - 1) / stride) <= Pm * Qm,
                    "conv_dgrad: the compact residual's phase must be the largest");
    } else {
      TORCH_CHECK(res->numel() == dx.numel(), "conv_dgrad: residual size mismatch");
    }
    TORCH_CHECK(dt16(*res, "res") == dt, "conv_dgrad: residual dtype");
    a.res = p16(*res, "res");
  }
  a.res_phase = (int)res_phase;
  a.N = N; a.H = P; a.W = Q; a.C = K; a.cs = K; a.Kout = C;
  a.ist_h = 1; a.ist_w = 1; a.tstep_h = -1; a.tstep_w = -1;
  a.OH = H; a.OW = W; a.ost_h = stride; a.ost_w = stride;
  a.nphase = (int)phases.size();
  int64_t maxM = 0;
  for (size_t i = 0; i < phases.size(); ++i) {
    const auto& f = phases[i];
    TORCH_CHECK(f.size() == 7, "conv_dgrad: phase = (ph, pw, T, U, ioff_h, ioff_w, woff)");
    const int64_t ph = f[0], pw = f[1];
    const int64_t Pm = (H - ph + stride - 1) / stride, Qm = (W - pw + stride - 1) / stride;
    TORCH_CHECK(Pm > 0 && Qm > 0 && f[6] + C * f[2] * f[3] * K <= wt.numel(), "conv_dgrad: bad phase");
    a.pooff_h[i] = (int)ph; a.pooff_w[i] = (int)pw; a.pT[i] = (int)f[2]; a.pU[i] = (int)f[3];
    a.pioff_h[i] = (int)f[4]; a.pioff_w[i] = (int)f[5]; a.pwoff[i] = f[6];
    a.pPm[i] = (int)Pm; a.pQm[i] = (int)Qm;
    maxM = std::max(maxM, N * Pm * Qm);
  }
  TORCH_CHECK(maxM < (int64_t(1) << 31), "conv_dgrad: N*Pm*Qm must be < 2^31 (32-bit pixel indexing)");
  a.M = maxM;
  if (bnb != 0) {
    // fused BN-backward reduce of the BatchNorm that consumes dx (see conv_fwd.h)
    TORCH_CHECK(bnb >= 1 && bnb <= 3, "conv_dgrad: bnb must be 0..3");
    TORCH_CHECK(bn_y1.has_value() && bn_coef1.has_value() && bn_slots.has_value(), "conv_dgrad: bnb needs y1/coef1/slots");
    TORCH_CHECK(bn_y1->numel() == dx.numel() && dt16(*bn_y1, "bn_y1") == dt && bn_coef1->numel() >= 4 * C,
                "conv_dgrad: bn_y1 / bn_coef1 size");
    TORCH_CHECK(bnb == 1 || bn_mask.has_value(), "conv_dgrad: bnb 2/3 need the block output's ReLU bitmask");
    TORCH_CHECK(bnb != 3 || (bn_y2.has_value() && bn_coef2.has_value() && bn_y2->numel() == dx.numel() &&
                             bn_coef2->numel() >= 4 * C),
                "conv_dgrad: bnb 3 needs y2/coef2");
    TORCH_CHECK((bnb == 1) == !res.has_value(), "conv_dgrad: bnb 1 runs without, 2/3 with the residual");
    TORCH_CHECK(C % 4 == 0 && bn_slots->numel() >= pdt::kStatSlots * C * (bnb == 3 ? 4 : 2),
                "conv_dgrad: bn_slots too small");
    a.bnb = (int)bnb;
    a.bn_y1 = p16(*bn_y1, "bn_y1");
    a.bn_coef1 = pf(*bn_coef1, "bn_coef1");
    if (bn_y2.has_value()) a.bn_y2 = p16(*bn_y2, "bn_y2");
    if (bn_coef2.has_value()) a.bn_coef2 = pf(*bn_coef2, "bn_coef2");
    a.bn_mask = pmask(bn_mask, dx.numel(), "bn_mask");
    a.stats = pd(*bn_slots, "bn_slots");
  }
  const int pk = dgrad_persistent_kind(K, C, bnb, stride, phases, H, W, P, Q, res_phase);
  if (pk == 1) {
    const auto& f = phases[0];
    {
      // 1x1 256 -> 64 | 128 conv's backward-data with the block-output BN-backward epilogue: persistent kernel
      // (conv1x1.hip);
      // its [256][K] weights start at the phase's offset (bounds checked with the phases above)
      pdt::conv1x1_c64_bnb_launch(a.x, a.w + f[6], a.y, a.res, a.bn_y1, a.bn_coef1, bnb == 3 ? a.bn_y2 : nullptr,
                                  bnb == 3 ? a.bn_coef2 : nullptr, a.bn_mask, a.stats, N * P * Q, (int)K, dt,
                                  cur_stream());
      launched("conv1x1_c64_bnb");
      return;
    }
  }
  if (pk == 2) {
    const auto& f = phases[0];
    {
      // ResNet-50 layers 2-4: 1x1 C -> 4C backward-data (conv1 of a bottleneck) with the block-output BN-backward
      // epilogue on the persistent sliced kernel (conv1x1x.hip); [C][K] weights at the phase's offset
      pdt::conv1x1x_bnb_launch(a.x, a.w + f[6], a.y, a.res, a.bn_y1, a.bn_coef1, bnb == 3 ? a.bn_y2 : nullptr,
                               bnb == 3 ? a.bn_coef2 : nullptr, a.bn_mask, a.stats, N * P * Q, (int)K, (int)C, dt,
                               cur_stream());
      launched("conv1x1x_bnb");
      return;
    }
  }
  pdt::conv_fwd_launch(a, dt, (int)bm, (int)bn, (int)bk, cur_stream());
  launched("conv_fwd_launch");
}

void conv_dgrad(const Tensor& dy, const Tensor& wt, Tensor& dx, const OptT& res, int64_t N, int64_t P, int64_t Q,
                int64_t K, int64_t C, int64_t H, int64_t W, int64_t stride, const std::vector<std::vector<int64_t>>& phases,
                int64_t bm, int64_t bn, int64_t bk) {
  conv_dgrad_impl(dy, wt, dx, res, N, P, Q, K, C, H, W, stride, phases, bm, bn, bk, 0, {}, {}, {}, {}, {}, {}, -1);
}

// 1x1 / stride-1 conv, 64 -> 256 channels, as the persistent store-overlapped kernel (conv1x1.hip): y[M][256] from
// x[M][64] and w[256][64], optional BN statistics (fp64 slots) of the rounded outputs
bool conv1x1_c64_supported(int64_t C, int64_t Kout) { return pdt::conv1x1_c64_supported((int)C, (int)Kout); }

// pre: the producer BN's [scale | shift] x 64 (x is its raw conv output; training forwards with statistics only)
void conv1x1_c64(const Tensor& x, const Tensor& w, Tensor& y, const OptT& stats, int64_t M, const OptT& pre) {
  const int dt = dt16(x, "x");
  TORCH_CHECK(dt16(w, "w") == dt && dt16(y, "y") == dt, "conv1x1_c64: mixed dtypes");
  TORCH_CHECK(x.numel() >= M * 64 && w.numel() == 256 * 64 && y.numel() >= M * 256, "conv1x1_c64: size mismatch");
  TORCH_CHECK(M * 256 < (int64_t(1) << 31), "conv1x1_c64: M*256 must be < 2^31 (32-bit buffer offsets)");
  double* st = nullptr;
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * 256 * 2, "conv1x1_c64: stats buffer too small");
    st = pd(*stats, "stats");
  }
  const float* pc = nullptr;
  if (pre.has_value()) {
    TORCH_CHECK(st != nullptr, "conv1x1_c64: a fused producer BN needs the statistics buffer (training forward)");
    TORCH_CHECK(pre->numel() >= 128, "conv1x1_c64: pre coefficients are [scale | shift] x 64");
    pc = pf(*pre, "pre");
  }
  pdt::conv1x1_c64_launch(p16(x, "x"), p16(w, "w"), p16(y, "y"), st, M, dt, cur_stream(), pc);
  launched("conv1x1_c64");
}

// 1x1 / stride-1 expanding conv with C = 128 / 256 / 512 input channels (ResNet-50 layers 2-4 conv3): the persistent
// sliced kernel (conv1x1x.hip); y[M][N] from x[M][C] and w[N][C], optional BN statistics (fp64 slots)
bool conv1x1x_supported(int64_t C, int64_t N) { return pdt::conv1x1x_supported((int)C, (int)N); }
int64_t conv1x1x_mode(int64_t set) { return pdt::conv1x1x_mode((int)set); }
int64_t conv1x1x_l1_mode(int64_t set) { return pdt::conv1x1x_l1_mode((int)set); }

// st > 1: stride-st 1x1 conv over nimg x H x W input images (M = nimg * P * Q)
void conv1x1x(const Tensor& x, const Tensor& w, Tensor& y, const OptT& stats, int64_t M, int64_t C, int64_t N,
              int64_t st, int64_t nimg, int64_t H, int64_t W) {
  const int dt = dt16(x, "x");
  TORCH_CHECK(dt16(w, "w") == dt && dt16(y, "y") == dt, "conv1x1x: mixed dtypes");
  TORCH_CHECK(pdt::conv1x1x_supported((int)C, (int)N), "conv1x1x: unsupported C / N (or PDT_CONV1X1X=0)");
  const int64_t xr = st > 1 ? nimg * H * W : M;
  TORCH_CHECK(st >= 1 && (st == 1 || nimg * ((H - 1) / st + 1) * ((W - 1) / st + 1) == M),
              "conv1x1x: strided geometry");
  TORCH_CHECK(x.numel() >= xr * C && w.numel() == N * C && y.numel() >= M * N, "conv1x1x: size mismatch");
  TORCH_CHECK(M * N < (int64_t(1) << 30) && M * C < (int64_t(1) << 30),
              "conv1x1x: operands exceed 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(xr * C < (int64_t(1) << 30), "conv1x1x: input exceeds 2 GiB (32-bit buffer offsets)");
  double* sp = nullptr;
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * N * 2, "conv1x1x: stats buffer too small");
    sp = pd(*stats, "stats");
  }
  pdt::conv1x1x_launch(p16(x, "x"), p16(w, "w"), p16(y, "y"), sp, M, (int)C, (int)N, dt, cur_stream(), (int)st,
                       (int)nimg, (int)H, (int)W);
  launched("conv1x1x");
}

std::vector<int64_t> conv_wgrad_plan(int64_t Kout, int64_t T, int64_t U, int64_t C, int64_t P, int64_t target_blocks,
                                     bool win) {
  pdt::ConvWgradArgs a{};
  a.Kout = Kout; a.T = T; a.U = U; a.C = C; a.P = P; a.win = win ? 1 : 0;
  pdt::conv_wgrad_plan(a, (int)target_blocks);
  return {a.splits, a.pix_per_split, a.tile};
}

void conv_wgrad(const Tensor& x, const Tensor& dy, Tensor& ws, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Kout,
                int64_t T, int64_t U, int64_t Pm, int64_t Qm, int64_t stride_h, int64_t stride_w, int64_t pad_h,
                int64_t pad_w, int64_t dil_h, int64_t dil_w, int64_t ldw, int64_t splits, int64_t pix_per_split,
                int64_t cs, bool win, const OptT& pre) {
  const int dt = dt16(x, "x");
  if (cs <= 0) cs = C;
  TORCH_CHECK(dt16(dy, "dy") == dt, "conv_wgrad: mixed dtypes");
  TORCH_CHECK(C % 64 == 0 && Kout % 64 == 0, "conv_wgrad: C and Kout must be multiples of 64");
  TORCH_CHECK(x.numel() == N * H * W * cs && dy.numel() == N * Pm * Qm * Kout, "conv_wgrad: size mismatch");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && dy.numel() < (int64_t(1) << 30),
              "conv_wgrad: operands exceed 2 GiB (32-bit buffer offsets)");
  if (win) {  // stem window mode: rows h..h+1 and 8 pixels from w must lie inside the padded image
    // U > 1: 8-pixel windows dil_w pixels apart (AlexNet's 11-wide kernel rows)
    TORCH_CHECK(cs == 4 && C == 64 && U >= 1 && dil_w >= 0 && pad_h == 0 && pad_w == 0 &&
                    (Pm - 1) * stride_h + (T - 1) * dil_h + 1 < H && ((Qm - 1) * stride_w + (U - 1) * dil_w + 8) <= W,
                "conv_wgrad: window-mode geometry leaves the padded image");
  } else {
    TORCH_CHECK(cs == C, "conv_wgrad: pixel stride must equal C outside window mode");
  }
  TORCH_CHECK(ldw >= T * U * C && ws.numel() >= splits * Kout * ldw, "conv_wgrad: workspace too small");
  pdt::ConvWgradArgs a{};
  a.x = p16(x, "x");
  a.dy = p16(dy, "dy");
  a.ws = pf(ws, "ws");
  a.N = N; a.H = H; a.W = W; a.C = C; a.Kout = Kout; a.T = T; a.U = U; a.Pm = Pm; a.Qm = Qm;
  a.stride_h = stride_h; a.stride_w = stride_w; a.pad_h = pad_h; a.pad_w = pad_w; a.dil_h = dil_h; a.dil_w = dil_w;
  a.P = N * Pm * Qm; a.ldw = ldw; a.splits = splits; a.pix_per_split = pix_per_split;
  a.cs = cs; a.win = win ? 1 : 0;
  a.tile = pdt::wgrad_tile((int)C, (int)Kout, win ? 1 : 0);
  TORCH_CHECK(pix_per_split % 128 == 0 && splits * pix_per_split >= a.P, "conv_wgrad: bad split plan");
  if (pre.has_value()) {  // x is the producer's raw output: its BN + ReLU applied in-kernel (1x1, C == 64)
    TORCH_CHECK(pre->numel() >= 2 * C && C == 64 && T == 1 && U == 1 && !win, "conv_wgrad: pre needs a 1x1 C=64 conv");
    a.pre_coef = pf(*pre, "pre");
  }
  pdt::conv_wgrad_launch(a, dt, cur_stream());
  launched("conv_wgrad_launch");
}

// ---------------------------------------------------------------------------- grouped convolution (ResNeXt)
// A grouped conv (groups g of cg channels, width = g * cg in and out) runs as width / S channel SLICES of S = 64:
// slice j is the dense S -> S conv of channels [j*S, (j+1)*S) with a block-diagonal weight (S / cg groups on the
// diagonal, zeros elsewhere: a derived layout gathered by the executor), on the generic implicit-GEMM kernels with
// strided operands (input pixel stride ``cs`` = width, output / BN-operand stride ``ldy`` = width, statistics slot
// row stride = the full width's).  The MFMA work is S / cg times the grouped FLOPs (16x at cg = 4 ... 2x at 32), in
// exchange for running on the tuned tiles with the fused statistics / BN-backward epilogues.
static constexpr int64_t kGSlice = 64;
#define PDT_BCOUNT(name)                                                  \
  do {                                                                    \
    static long long* _c = pdt::dispatch_counter(name);                   \
    __atomic_fetch_add(_c, 1LL, __ATOMIC_RELAXED);                        \
  } while (0)

void gconv_fwd(const Tensor& x, const Tensor& wslice, Tensor& y, const OptT& stats, int64_t N, int64_t H, int64_t W,
               int64_t width, int64_t R, int64_t stride, int64_t pad, int64_t P, int64_t Q, int64_t j, int64_t bm,
               int64_t bn) {
  const int dt = dt16(x, "x");
  const int64_t S = kGSlice;
  TORCH_CHECK(dt16(wslice, "w") == dt && dt16(y, "y") == dt, "gconv_fwd: mixed dtypes");
  // j == -1: every slice in ONE launch (ConvFwdArgs::nslice; wslice = the slices' layouts back to back)
  TORCH_CHECK(width % S == 0 && j >= -1 && j < width / S, "gconv_fwd: bad slice");
  const int64_t nsl = j < 0 ? width / S : 1;
  TORCH_CHECK(x.numel() == N * H * W * width && y.numel() == N * P * Q * width && wslice.numel() == nsl * S * R * R * S,
              "gconv_fwd: size mismatch");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && y.numel() < (int64_t(1) << 30), "gconv_fwd: operands exceed 2 GiB");
  TORCH_CHECK(S % bn == 0 && N * P * Q < (int64_t(1) << 31), "gconv_fwd: tile / size");
  pdt::ConvFwdArgs a{};
  const int64_t j0 = j < 0 ? 0 : j;
  a.x = p16(x, "x") + j0 * S;
  a.w = p16(wslice, "w");
  a.y = p16(y, "y") + j0 * S;
  if (j < 0) {
    a.nslice = (int)nsl;
    a.slice_wstride = S * R * R * S;
  }
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * width * 2, "gconv_fwd: stats buffer too small");
    a.stats = pd(*stats, "stats") + j0 * S * 2;
    a.stats_ld = (int)(width * 2);
  }
  a.N = N; a.H = H; a.W = W; a.C = S; a.Kout = S; a.T = R; a.U = R; a.Pm = P; a.Qm = Q; a.cs = width;
  a.ldy = (int)width;
  a.ist_h = stride; a.ist_w = stride; a.ioff_h = -pad; a.ioff_w = -pad; a.tstep_h = 1; a.tstep_w = 1;
  a.OH = P; a.OW = Q; a.ost_h = 1; a.ost_w = 1; a.ooff_h = 0; a.ooff_w = 0;
  a.M = N * P * Q;
  pdt::conv_fwd_launch(a, dt, (int)bm, (int)bn, 64, cur_stream());
  launched("gconv_fwd");
  PDT_BCOUNT("gconv_fwd");
}

// backward data of slice j (phases and their derived-weight offsets as conv_dgrad), optionally with the fused
// reduce of the BatchNorm + ReLU that produced the conv's input (bnb 1: y1 / coef1 / slots of the full width)
void gconv_dgrad(const Tensor& dy, const Tensor& wt, Tensor& dx, int64_t N, int64_t P, int64_t Q, int64_t width,
                 int64_t H, int64_t W, int64_t stride, const std::vector<std::vector<int64_t>>& phases, int64_t j,
                 int64_t bm, int64_t bn, const OptT& bn_y1, const OptT& bn_coef1, const OptT& bn_slots) {
  const int dt = dt16(dy, "dy");
  const int64_t S = kGSlice;
  TORCH_CHECK(dt16(wt, "wt") == dt && dt16(dx, "dx") == dt, "gconv_dgrad: mixed dtypes");
  TORCH_CHECK(width % S == 0 && j >= -1 && j < width / S, "gconv_dgrad: bad slice");  // -1: every slice, one launch
  const int64_t j0 = j < 0 ? 0 : j, nsl = j < 0 ? width / S : 1;
  int64_t taps = 0;  // every phase's taps together: one slice's R x R
  for (const auto& f : phases) taps += f.size() == 7 ? f[2] * f[3] : 0;
  const int64_t wstride = S * S * taps;  // elements of one slice's derived phase weights
  TORCH_CHECK(dy.numel() == N * P * Q * width && dx.numel() == N * H * W * width, "gconv_dgrad: size mismatch");
  TORCH_CHECK(dy.numel() < (int64_t(1) << 30) && dx.numel() < (int64_t(1) << 30), "gconv_dgrad: operands exceed 2 GiB");
  TORCH_CHECK(!phases.empty() && phases.size() <= 4 && S % bn == 0, "gconv_dgrad: 1..4 phases / tile");
  pdt::ConvFwdArgs a{};
  a.x = p16(dy, "dy") + j0 * S;
  a.w = p16(wt, "wt");
  a.y = p16(dx, "dx") + j0 * S;
  if (j < 0) {
    a.nslice = (int)nsl;
    a.slice_wstride = wstride;
  }
  a.N = N; a.H = P; a.W = Q; a.C = S; a.cs = width; a.Kout = S; a.ldy = (int)width;
  a.ist_h = 1; a.ist_w = 1; a.tstep_h = -1; a.tstep_w = -1;
  a.OH = H; a.OW = W; a.ost_h = stride; a.ost_w = stride;
  a.nphase = (int)phases.size();
  a.res_phase = -1;
  int64_t maxM = 0;
  for (size_t i = 0; i < phases.size(); ++i) {
    const auto& f = phases[i];
    TORCH_CHECK(f.size() == 7, "gconv_dgrad: phase = (ph, pw, T, U, ioff_h, ioff_w, woff)");
    const int64_t ph = f[0], pw = f[1];
    const int64_t Pm = (H - ph + stride - 1) / stride, Qm = (W - pw + stride - 1) / stride;
    TORCH_CHECK(Pm > 0 && Qm > 0 && f[6] + S * f[2] * f[3] * S + (nsl - 1) * wstride <= wt.numel(),
                "gconv_dgrad: bad phase");
    a.pooff_h[i] = (int)ph; a.pooff_w[i] = (int)pw; a.pT[i] = (int)f[2]; a.pU[i] = (int)f[3];
    a.pioff_h[i] = (int)f[4]; a.pioff_w[i] = (int)f[5]; a.pwoff[i] = f[6];
    a.pPm[i] = (int)Pm; a.pQm[i] = (int)Qm;
    maxM = std::max(maxM, N * Pm * Qm);
  }
  TORCH_CHECK(maxM < (int64_t(1) << 31), "gconv_dgrad: 32-bit pixel indexing");
  a.M = maxM;
  if (bn_y1.has_value()) {  // bnb 1: ReLU mask from y1 and the forward coefficients; dx holds dz
    TORCH_CHECK(bn_coef1.has_value() && bn_slots.has_value() && bn_y1->numel() == dx.numel() &&
                    dt16(*bn_y1, "bn_y1") == dt && bn_coef1->numel() >= 4 * width &&
                    bn_slots->numel() >= pdt::kStatSlots * width * 2,
                "gconv_dgrad: bnb needs y1 / coef1 (4 x width) / slots of the full width");
    a.bnb = 1;
    a.bn_y1 = p16(*bn_y1, "bn_y1") + j0 * S;
    a.bn_coef1 = pf(*bn_coef1, "bn_coef1") + j0 * S;
    a.coef_ld = (int)width;
    a.stats = pd(*bn_slots, "bn_slots") + j0 * S * 2;
    a.stats_ld = (int)(width * 2);
  }
  pdt::conv_fwd_launch(a, dt, (int)bm, (int)bn, 64, cur_stream());
  launched("gconv_dgrad");
  PDT_BCOUNT("gconv_dgrad");
}

// weight gradient of slice j: the dense S x (R*R*S) partials [splits][S][ldw] (the executor keeps the diagonal blocks)
void gconv_wgrad(const Tensor& x, const Tensor& dy, Tensor& ws, int64_t N, int64_t H, int64_t W, int64_t width,
                 int64_t R, int64_t P, int64_t Q, int64_t stride, int64_t pad, int64_t j, int64_t ldw, int64_t splits,
                 int64_t pix_per_split) {
  const int dt = dt16(x, "x");
  const int64_t S = kGSlice;
  TORCH_CHECK(dt16(dy, "dy") == dt, "gconv_wgrad: mixed dtypes");
  TORCH_CHECK(width % S == 0 && j >= -1 && j < width / S, "gconv_wgrad: bad slice");  // -1: every slice, one launch
  const int64_t j0 = j < 0 ? 0 : j, nsl = j < 0 ? width / S : 1;
  TORCH_CHECK(x.numel() == N * H * W * width && dy.numel() == N * P * Q * width, "gconv_wgrad: size mismatch");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && dy.numel() < (int64_t(1) << 30), "gconv_wgrad: operands exceed 2 GiB");
  TORCH_CHECK(ldw >= R * R * S && ws.numel() >= splits * nsl * S * ldw, "gconv_wgrad: workspace too small");
  pdt::ConvWgradArgs a{};
  a.x = p16(x, "x") + j0 * S;
  a.dy = p16(dy, "dy") + j0 * S;
  if (j < 0) a.nslice = (int)nsl;
  a.ws = pf(ws, "ws");
  a.N = N; a.H = H; a.W = W; a.C = S; a.Kout = S; a.T = R; a.U = R; a.Pm = P; a.Qm = Q;
  a.stride_h = stride; a.stride_w = stride; a.pad_h = pad; a.pad_w = pad; a.dil_h = 1; a.dil_w = 1;
  a.P = N * P * Q; a.ldw = ldw; a.splits = splits; a.pix_per_split = pix_per_split;
  a.cs = width; a.ldy = (int)width; a.win = 0;
  a.tile = pdt::wgrad_tile((int)S, (int)S, 0);
  TORCH_CHECK(a.tile == 64 && pix_per_split % 128 == 0 && splits * pix_per_split >= a.P, "gconv_wgrad: bad plan");
  pdt::conv_wgrad_launch(a, dt, cur_stream());
  launched("gconv_wgrad");
  PDT_BCOUNT("gconv_wgrad");
}

// ResNet stem weight gradient with its dY computed in-kernel (max-pool backward + ReLU mask + BN-backward
// apply from the pooled gradient dp, the argmax idx, the conv output y0 and the BN coefficients): the
// window-mode conv_wgrad above without the [P][64] dY tensor.  x: padded NHWC4 image [N][Hp][Wp][4].
void conv_wgrad_stem_fused(const Tensor& x, const Tensor& dp, const Tensor& idx, const Tensor& y0, const Tensor& coef,
                           const Tensor& bcoef, Tensor& ws, int64_t N, int64_t Hp, int64_t Wp, int64_t pairs,
                           int64_t Pm, int64_t Qm, int64_t stride, int64_t dil, int64_t ldw, int64_t splits,
                           int64_t pix_per_split) {
  const int dt = dt16(x, "x");
  const int64_t OH = (Pm - 1) / 2 + 1, OW = (Qm - 1) / 2 + 1;  // 3x3/2 pad-1 max-pool output
  TORCH_CHECK(dt16(dp, "dp") == dt && dt16(y0, "y0") == dt, "conv_wgrad_stem_fused: mixed dtypes");
  TORCH_CHECK(x.numel() == N * Hp * Wp * 4 && y0.numel() == N * Pm * Qm * 64 && dp.numel() == N * OH * OW * 64 &&
                  idx.numel() == dp.numel() && coef.numel() >= 2 * 64 && bcoef.numel() >= 3 * 64,
              "conv_wgrad_stem_fused: size mismatch");
  TORCH_CHECK(Qm % 2 == 0, "conv_wgrad_stem_fused: the conv output width must be even (pixel pairs)");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && N * Pm * Qm * 64 < (int64_t(1) << 31),
              "conv_wgrad_stem_fused: operands exceed 32-bit offsets");
  TORCH_CHECK(pairs == 4 && ldw >= 256 && ws.numel() >= splits * 64 * ldw, "conv_wgrad_stem_fused: needs 4 row pairs");
  TORCH_CHECK((Pm - 1) * stride + (pairs - 1) * dil + 1 < Hp && ((Qm - 1) * stride + 8) <= Wp,
              "conv_wgrad_stem_fused: window-mode geometry leaves the padded image");
  check_dev(idx, "idx");
  pdt::ConvWgradArgs a{};
  a.x = p16(x, "x");
  a.dy = nullptr;
  a.ws = pf(ws, "ws");
  a.N = N; a.H = Hp; a.W = Wp; a.C = 64; a.Kout = 64; a.T = pairs; a.U = 1; a.Pm = Pm; a.Qm = Qm;
  a.stride_h = stride; a.stride_w = stride; a.pad_h = 0; a.pad_w = 0; a.dil_h = dil; a.dil_w = dil;
  a.P = N * Pm * Qm; a.ldw = ldw; a.splits = splits; a.pix_per_split = pix_per_split;
  a.cs = 4; a.win = 1;
  a.tile = pdt::wgrad_tile(64, 64, 1);
  TORCH_CHECK(pix_per_split % 128 == 0 && splits * pix_per_split >= a.P, "conv_wgrad_stem_fused: bad split plan");
  {  // the kernel walks pixels in 2x2 quads: an odd height pads the count to whole quads (same splits, same ws)
    const int64_t pq = N * ((Pm + 1) / 2) * 2 * Qm;
    if (splits * a.pix_per_split < pq) a.pix_per_split = (int)(((pq + splits - 1) / splits + 127) / 128 * 128);
  }
  a.f_y = p16(y0, "y0");
  a.f_dp = p16(dp, "dp");
  a.f_idx = idx.data_ptr<uint8_t>();
  a.f_coef = pf(coef, "coef");
  a.f_bcoef = pf(bcoef, "bcoef");
  a.f_OH = (int)OH; a.f_OW = (int)OW;
  pdt::conv_wgrad_launch(a, dt, cur_stream());
  launched("conv_wgrad_launch");
}

// ResNet layer1 weight gradient (3x3/s1/p1, C = Kout = 64, W = 56): all 9 taps per block; writes at most
// wgrad_blocks_3x3c64() fp32 partials [.][64][576] into ws and returns how many it wrote (sum them with wgrad_reduce).
int64_t wgrad_blocks_3x3c64() { return pdt::wgrad3x3_c64_blocks(); }

bool wgrad_3x3c64_supported(int64_t C, int64_t Kout, int64_t T, int64_t U, int64_t W, int64_t stride, int64_t pad) {
  return pdt::wgrad3x3_c64_supported((int)C, (int)Kout, (int)T, (int)U, (int)W, (int)stride, (int)pad, 0);
}

int64_t conv_wgrad_3x3c64(const Tensor& x, const Tensor& dy, Tensor& ws, int64_t N, int64_t H, int64_t W,
                          const OptT& pre_coef) {
  const int dt = dt16(x, "x");
  TORCH_CHECK(dt16(dy, "dy") == dt, "conv_wgrad_3x3c64: mixed dtypes");
  TORCH_CHECK(pdt::wgrad3x3_c64_supported(64, 64, 3, 3, (int)W, 1, 1, 0), "conv_wgrad_3x3c64: needs W == 56");
  TORCH_CHECK(x.numel() == N * H * W * 64 && dy.numel() == x.numel(), "conv_wgrad_3x3c64: size mismatch");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30), "conv_wgrad_3x3c64: operands exceed 2 GiB (32-bit buffer offsets)");
  const int blocks = pdt::wgrad3x3_c64_blocks();
  TORCH_CHECK(ws.numel() >= (int64_t)blocks * 64 * 576, "conv_wgrad_3x3c64: workspace too small");
  pdt::ConvWgradArgs a{};
  a.x = p16(x, "x");
  a.dy = p16(dy, "dy");
  a.ws = pf(ws, "ws");
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.C = 64; a.Kout = 64; a.T = 3; a.U = 3; a.ldw = 576;
  if (pre_coef.has_value()) {
    TORCH_CHECK(pre_coef->numel() >= 128, "conv_wgrad_3x3c64: pre_coef needs scale[64] | shift[64]");
    a.pre_coef = pf(*pre_coef, "pre_coef");
  }
  const int written = pdt::wgrad3x3_c64_launch(a, blocks, dt, cur_stream());
  launched("wgrad3x3_c64_launch");
  return written;
}

// grouped conv weight gradient of every 64-channel slice on the layer1 halo kernel (ResNeXt stage 1: 3x3 / s1 / p1,
// W = 56): partials [parts][nslice][64][576] (returns parts; wgrad_reduce over nslice * 64 rows sums them)
int64_t gconv_wgrad_l1(const Tensor& x, const Tensor& dy, Tensor& ws, int64_t N, int64_t H, int64_t W, int64_t width) {
  const int dt = dt16(x, "x");
  const int64_t S = kGSlice, nsl = width / S;
  TORCH_CHECK(dt16(dy, "dy") == dt, "gconv_wgrad_l1: mixed dtypes");
  TORCH_CHECK(width % S == 0 && pdt::wgrad3x3_c64_supported(64, 64, 3, 3, (int)W, 1, 1, 0), "gconv_wgrad_l1: geometry");
  TORCH_CHECK(x.numel() == N * H * W * width && dy.numel() == x.numel(), "gconv_wgrad_l1: size mismatch");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30), "gconv_wgrad_l1: operands exceed 2 GiB (32-bit buffer offsets)");
  const int blocks = pdt::wgrad3x3_c64_blocks();
  TORCH_CHECK(ws.numel() >= (int64_t)blocks * nsl * 64 * 576, "gconv_wgrad_l1: workspace too small");
  int written = 0;
  for (int64_t j = 0; j < nsl; ++j) {
    pdt::ConvWgradArgs a{};
    a.x = p16(x, "x") + j * S;
    a.dy = p16(dy, "dy") + j * S;
    a.ws = pf(ws, "ws") + j * S * 576;
    a.N = (int)N; a.H = (int)H; a.W = (int)W; a.C = 64; a.Kout = 64; a.T = 3; a.U = 3; a.ldw = 576;
    a.cs = (int)width; a.ldy = (int)width; a.nslice = (int)nsl;
    written = pdt::wgrad3x3_c64_launch(a, blocks, dt, cur_stream());
  }
  launched("gconv_wgrad_l1");
  PDT_BCOUNT("gconv_wgrad_l1");
  return written;
}

void wgrad_reduce(const Tensor& ws, int64_t splits, int64_t rows, int64_t cols, int64_t ldw, int64_t split_stride,
                  Tensor& out, int64_t ldo, double scale, bool accumulate) {
  TORCH_CHECK(ws.numel() >= (splits - 1) * split_stride + (rows - 1) * ldw + cols, "wgrad_reduce: ws too small");
  TORCH_CHECK(out.numel() >= (rows - 1) * ldo + cols, "wgrad_reduce: out too small");
  pdt::wgrad_reduce_launch(pf(ws, "ws"), splits, rows, cols, ldw, split_stride, pf(out, "out"), ldo, (float)scale,
                           accumulate, cur_stream());
  launched("wgrad_reduce_launch");
}

// -------------------------------------------------------------------------------------------- bn
void bn_slot_sum(const Tensor& slots, int64_t C, int64_t K, Tensor& sums) {
  TORCH_CHECK(slots.numel() >= pdt::kStatSlots * C * K && sums.numel() >= C * K, "bn_slot_sum: bad sizes");
  pdt::bn_slot_sum_launch(pd(slots, "slots"), C, K, pd(sums, "sums"), cur_stream());
  launched("bn_slot_sum_launch");
}

int64_t stat_slots() { return pdt::kStatSlots; }

// slot sum + finalize in one launch (no SyncBN): slots [kStatSlots][C][2] -> coef (+ running stats), sums
void bn_finalize_slots(const Tensor& slots, double count, const Tensor& gamma, const Tensor& beta, double eps,
                       double momentum, Tensor& rm, Tensor& rv, Tensor& coef, Tensor& sums, bool update_running) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(slots.numel() >= pdt::kStatSlots * C * 2 && coef.numel() >= 4 * C && sums.numel() >= 2 * C,
              "bn_finalize_slots: bad sizes");
  pdt::bn_finalize_slots_launch(pd(slots, "slots"), count, pf(gamma, "gamma"), pf(beta, "beta"), (float)eps,
                                (float)momentum, pf(rm, "running_mean"), pf(rv, "running_var"), pf(coef, "coef"),
                                pd(sums, "sums"), (int)C, update_running, cur_stream());
  launched("bn_finalize_slots_launch");
}

// slot sum + backward finalize for one (K = 2) or two (K = 4) BN branches, no SyncBN
void bn_bwd_finalize_slots(const Tensor& slots, int64_t K, double count, const Tensor& coef1, const Tensor& gamma1,
                           const OptT& dgamma1, const OptT& dbeta1, Tensor& bcoef1, const OptT& coef2,
                           const OptT& gamma2, const OptT& dgamma2, const OptT& dbeta2, const OptT& bcoef2,
                           double gscale) {
  const int64_t C = gamma1.numel();
  TORCH_CHECK((K == 2 || K == 4) && slots.numel() >= pdt::kStatSlots * C * K && bcoef1.numel() >= 3 * C,
              "bn_bwd_finalize_slots: bad sizes");
  TORCH_CHECK(K == 2 || (coef2.has_value() && gamma2.has_value() && bcoef2.has_value() && bcoef2->numel() >= 3 * C),
              "bn_bwd_finalize_slots: K == 4 needs the second branch");
  pdt::bn_bwd_finalize_slots_launch(pd(slots, "slots"), (int)K, count, pf(coef1, "coef1"), pf(gamma1, "gamma1"),
                                    pfo(dgamma1, "dgamma1"), pfo(dbeta1, "dbeta1"), pf(bcoef1, "bcoef1"),
                                    pfo(coef2, "coef2"), pfo(gamma2, "gamma2"), pfo(dgamma2, "dgamma2"),
                                    pfo(dbeta2, "dbeta2"), pfo(bcoef2, "bcoef2"), (float)gscale, (int)C,
                                    cur_stream());
  launched("bn_bwd_finalize_slots_launch");
}

void bn_finalize(const Tensor& sums, double count, const Tensor& gamma, const Tensor& beta, double eps, double momentum,
                 Tensor& rm, Tensor& rv, Tensor& coef, bool update_running) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(coef.numel() >= 4 * C && sums.numel() >= 2 * C, "bn_finalize: size mismatch");
  pdt::bn_finalize_launch(pd(sums, "sums"), count, pf(gamma, "gamma"), pf(beta, "beta"), (float)eps, (float)momentum,
                          pf(rm, "running_mean"), pf(rv, "running_var"), pf(coef, "coef"), C, update_running,
                          cur_stream());
  launched("bn_finalize_launch");
}

void bn_eval_coef(const Tensor& gamma, const Tensor& beta, const Tensor& rm, const Tensor& rv, double eps, Tensor& coef) {
  const int64_t C = gamma.numel();
  pdt::bn_eval_coef_launch(pf(gamma, "gamma"), pf(beta, "beta"), pf(rm, "rm"), pf(rv, "rv"), (float)eps, pf(coef, "coef"),
                           C, cur_stream());
  launched("bn_eval_coef_launch");
}

void bn_apply(const Tensor& y, const Tensor& coef, const OptT& res, const OptT& rcoef, Tensor& out, int64_t C,
              int64_t resmode, bool relu, const OptT& mask) {
  const int dt = dt16(y, "y");
  TORCH_CHECK(C % 8 == 0 && y.numel() % C == 0 && out.numel() == y.numel(), "bn_apply: bad sizes");
  if (resmode != 0) TORCH_CHECK(res.has_value() && res->numel() == y.numel(), "bn_apply: residual missing/mismatch");
  if (resmode == 2) TORCH_CHECK(rcoef.has_value(), "bn_apply: residual coefficients missing");
  TORCH_CHECK(!mask.has_value() || (resmode != 0 && relu), "bn_apply: the ReLU bitmask is built for residual block outputs");
  pdt::bn_apply_launch(dt, p16(y, "y"), pf(coef, "coef"), p16o(res, "res"), pfo(rcoef, "rcoef"), p16(out, "out"),
                       pmask(mask, y.numel(), "mask"), y.numel(), C, (int)resmode, relu, cur_stream());
  launched("bn_apply_launch");
}

int64_t bn_bwd_reduce_blocks(int64_t rows, int64_t C) { return pdt::bn_bwd_reduce_blocks(rows, (int)C); }

void bn_bwd_reduce(const Tensor& g, const OptT& mask, const Tensor& y1, const Tensor& coef1, const OptT& y2,
                   const OptT& coef2, Tensor& slots, int64_t blocks, int64_t rows, int64_t C) {
  const int dt = dt16(g, "g");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && g.numel() == rows * C && y1.numel() == rows * C, "bn_bwd_reduce: bad sizes");
  const int K = y2.has_value() ? 4 : 2;
  TORCH_CHECK(slots.numel() >= pdt::kStatSlots * C * K, "bn_bwd_reduce: slots too small");
  pdt::bn_bwd_reduce_launch(dt, p16(g, "g"), pmask(mask, g.numel(), "mask"), p16(y1, "y1"), pf(coef1, "coef1"), p16o(y2, "y2"),
                            pfo(coef2, "coef2"), pd(slots, "slots"), (int)blocks, rows, (int)C, cur_stream());
  launched("bn_bwd_reduce_launch");
}

void bn_bwd_finalize(const Tensor& sums, double count, const Tensor& coef, const Tensor& gamma, const OptT& dgamma,
                     const OptT& dbeta, double gscale, Tensor& bcoef) {
  const int64_t C = gamma.numel();
  TORCH_CHECK(bcoef.numel() >= 3 * C, "bn_bwd_finalize: bcoef too small");
  pdt::bn_bwd_finalize_launch(pd(sums, "sums"), count, pf(coef, "coef"), pf(gamma, "gamma"), pfo(dgamma, "dgamma"),
                              pfo(dbeta, "dbeta"), (float)gscale, pf(bcoef, "bcoef"), C, cur_stream());
  launched("bn_bwd_finalize_launch");
}

void bn_bwd_apply(const Tensor& g, const OptT& mask, const Tensor& y1, const Tensor& b1, Tensor& dy1, const OptT& y2,
                  const OptT& b2, const OptT& dy2, const OptT& dz, int64_t C) {
  const int dt = dt16(g, "g");
  TORCH_CHECK(C % 8 == 0 && g.numel() % C == 0 && dy1.numel() == g.numel(), "bn_bwd_apply: bad sizes");
  pdt::bn_bwd_apply_launch(dt, p16(g, "g"), pmask(mask, g.numel(), "mask"), p16(y1, "y1"), pf(b1, "b1"), p16(dy1, "dy1"),
                           p16o(y2, "y2"), pfo(b2, "b2"), p16m(dy2, "dy2"), p16m(dz, "dz"), g.numel(), C, cur_stream());
  launched("bn_bwd_apply_launch");
}

// ------------------------------------------------------------------------------------------ pool
// MaxPool(3, 2, pad): pad 1 (ResNet stem) or 0 (AlexNet)
void bn_relu_maxpool(const Tensor& y, const Tensor& coef, Tensor& out, Tensor& idx, int64_t N, int64_t H, int64_t W,
                     int64_t C, int64_t pad) {
  const int dt = dt16(y, "y");
  TORCH_CHECK((pad == 0 || pad == 1) && H + 2 * pad >= 3 && W + 2 * pad >= 3, "bn_relu_maxpool: pad 0 or 1");
  const int64_t OH = (H + 2 * pad - 3) / 2 + 1, OW = (W + 2 * pad - 3) / 2 + 1;
  TORCH_CHECK(y.numel() == N * H * W * C && out.numel() == N * OH * OW * C && idx.numel() == out.numel() && C % 8 == 0,
              "bn_relu_maxpool: bad sizes");
  TORCH_CHECK(y.numel() < (int64_t(1) << 32), "bn_relu_maxpool: tensor exceeds 2^32 elements (32-bit indexing)");
  check_dev(idx, "idx");
  pdt::bn_relu_maxpool_launch(dt, p16(y, "y"), pf(coef, "coef"), p16(out, "out"), idx.data_ptr<uint8_t>(), N, H, W, C,
                              cur_stream(), (int)pad);
  launched("bn_relu_maxpool_launch");
}

void maxpool_bwd_relu(const Tensor& dp, const Tensor& idx, const Tensor& y, const Tensor& coef, Tensor& dz, int64_t N,
                      int64_t H, int64_t W, int64_t C, int64_t pad) {
  const int dt = dt16(dp, "dp");
  TORCH_CHECK((pad == 0 || pad == 1) && H + 2 * pad >= 3 && W + 2 * pad >= 3 && C % 8 == 0,
              "maxpool_bwd_relu: pad 0 or 1, C % 8 == 0");
  const int64_t OH = (H + 2 * pad - 3) / 2 + 1, OW = (W + 2 * pad - 3) / 2 + 1;
  TORCH_CHECK(dp.numel() == N * OH * OW * C && y.numel() == N * H * W * C && dz.numel() == y.numel(),
              "maxpool_bwd_relu: bad sizes");
  check_dev(idx, "idx");
  pdt::maxpool_bwd_relu_launch(dt, p16(dp, "dp"), idx.data_ptr<uint8_t>(), p16(y, "y"), pf(coef, "coef"), p16(dz, "dz"),
                               N, H, W, C, cur_stream(), (int)pad);
  launched("maxpool_bwd_relu_launch");
}

// Stem backward (max-pool bwd + ReLU mask + BN bwd) without the 112x112 dz tensor: reduce pass ...
void stem_pool_bwd_reduce(const Tensor& dp, const Tensor& idx, const Tensor& y, const Tensor& coef, Tensor& slots,
                          int64_t N, int64_t H, int64_t W, int64_t C) {
  const int dt = dt16(dp, "dp");
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dt16(y, "y") == dt && dp.numel() == N * OH * OW * C && y.numel() == N * H * W * C &&
                  idx.numel() == dp.numel() && C % 8 == 0 && C <= 2048 && coef.numel() >= 4 * C,
              "stem_pool_bwd_reduce: bad sizes");
  TORCH_CHECK(slots.numel() >= pdt::kStatSlots * C * 2, "stem_pool_bwd_reduce: slots too small");
  check_dev(idx, "idx");
  pdt::stem_pool_bwd_reduce_launch(dt, p16(dp, "dp"), idx.data_ptr<uint8_t>(), p16(y, "y"), pf(coef, "coef"),
                                   pd(slots, "slots"), N, H, W, C, cur_stream());
  launched("stem_pool_bwd_reduce_launch");
}

// pass 1 from the pooled output alone (mask = out > 0, BN input recovered from out)
void stem_pool_bwd_reduce_out(const Tensor& dp, const Tensor& out, const Tensor& coef, Tensor& slots, int64_t N,
                              int64_t H, int64_t W, int64_t C) {
  const int dt = dt16(dp, "dp");
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dt16(out, "out") == dt && dp.numel() == N * OH * OW * C && out.numel() == dp.numel() && C % 8 == 0 &&
                  C <= 2048 && coef.numel() >= 4 * C,
              "stem_pool_bwd_reduce_out: bad sizes");
  TORCH_CHECK(slots.numel() >= pdt::kStatSlots * C * 2, "stem_pool_bwd_reduce_out: slots too small");
  pdt::stem_pool_bwd_reduce_out_launch(dt, p16(dp, "dp"), p16(out, "out"), pf(coef, "coef"), pd(slots, "slots"), N, H,
                                       W, C, cur_stream());
  launched("stem_pool_bwd_reduce_out_launch");
}

// ---------------------------------------------------------------------------- VGG family (vgg.hip)
// out = MaxPool(2, 2)(relu(y * coef[0:C] + coef[C:2C])), idx = window argmax (0..3) per pooled element (training)
void bn_relu_maxpool2(const Tensor& y, const Tensor& coef, Tensor& out, const OptT& idx, int64_t N, int64_t H,
                      int64_t W, int64_t C) {
  const int dt = dt16(y, "y");
  TORCH_CHECK(dt16(out, "out") == dt && H % 2 == 0 && W % 2 == 0 && C % 8 == 0 && coef.numel() >= 2 * C &&
                  y.numel() == N * H * W * C && out.numel() == N * (H / 2) * (W / 2) * C,
              "bn_relu_maxpool2: bad sizes (even H, W; C % 8 == 0)");
  TORCH_CHECK(!idx.has_value() || (idx->scalar_type() == at::kByte && idx->numel() == out.numel()),
              "bn_relu_maxpool2: idx must be uint8 like out");
  pdt::bn_relu_maxpool2_launch(dt, p16(y, "y"), pf(coef, "coef"), p16(out, "out"),
                               idx.has_value() ? idx->data_ptr<uint8_t>() : nullptr, N, (int)H, (int)W, (int)C,
                               cur_stream());
  launched("bn_relu_maxpool2_launch");
}

// dy (conv output gradient) of a BN / bias + ReLU + MaxPool(2, 2): bcoef given -> dy = A*dz + B*y + C, else dz
void maxpool2_bwd(const Tensor& dp, const Tensor& idx, const Tensor& out, const OptT& y, const OptT& bcoef,
                  Tensor& dy, int64_t N, int64_t H, int64_t W, int64_t C) {
  const int dt = dt16(dp, "dp");
  TORCH_CHECK(dt16(out, "out") == dt && dt16(dy, "dy") == dt && H % 2 == 0 && W % 2 == 0 && C % 8 == 0 &&
                  dp.numel() == N * (H / 2) * (W / 2) * C && out.numel() == dp.numel() && idx.numel() == dp.numel() &&
                  idx.scalar_type() == at::kByte && dy.numel() == N * H * W * C,
              "maxpool2_bwd: bad sizes");
  TORCH_CHECK(bcoef.has_value() == y.has_value() && (!y.has_value() || (dt16(*y, "y") == dt && y->numel() == dy.numel())) &&
                  (!bcoef.has_value() || bcoef->numel() >= 3 * C),
              "maxpool2_bwd: a BatchNorm needs both y and bcoef");
  pdt::maxpool2_bwd_launch(dt, p16(dp, "dp"), idx.data_ptr<uint8_t>(), p16(out, "out"), p16o(y, "y"), pfo(bcoef, "bcoef"),
                           p16(dy, "dy"), N, (int)H, (int)W, (int)C, cur_stream());
  launched("maxpool2_bwd_launch");
}

// BN-backward sums (sum dz, sum dz * xhat) of any max-pool over relu(BN(y)) from the pooled tensors alone
void pooled_bwd_reduce(const Tensor& dp, const Tensor& out, const Tensor& coef, Tensor& slots, int64_t rows, int64_t C) {
  const int dt = dt16(dp, "dp");
  TORCH_CHECK(dt16(out, "out") == dt && dp.numel() == rows * C && out.numel() == dp.numel() && C % 8 == 0 &&
                  C <= 2048 && coef.numel() >= 4 * C && slots.numel() >= pdt::kStatSlots * C * 2,
              "pooled_bwd_reduce: bad sizes");
  pdt::pooled_bwd_reduce_launch(dt, p16(dp, "dp"), p16(out, "out"), pf(coef, "coef"), pd(slots, "slots"), rows, (int)C,
                                cur_stream());
  launched("pooled_bwd_reduce_launch");
}

// classifier: out = dropout_p(relu(z + bias)) (seed: a fresh value per step); p = 0: bias + ReLU only
void fc_act_fwd(const Tensor& z, const Tensor& bias, Tensor& out, int64_t rows, int64_t F, double p, int64_t seed) {
  const int dt = dt16(z, "z");
  TORCH_CHECK(dt16(out, "out") == dt && F % 8 == 0 && z.numel() == rows * F && out.numel() == z.numel() &&
                  bias.numel() >= F && p >= 0.0 && p < 1.0,
              "fc_act_fwd: bad sizes");
  pdt::fc_act_fwd_launch(dt, p16(z, "z"), pf(bias, "bias"), p16(out, "out"), rows, (int)F, p, (uint64_t)seed,
                         cur_stream());
  launched("fc_act_fwd_launch");
}

void fc_act_bwd(const Tensor& dh, const Tensor& out, Tensor& dz, double p) {
  const int dt = dt16(dh, "dh");
  TORCH_CHECK(dt16(out, "out") == dt && dt16(dz, "dz") == dt && dh.numel() == out.numel() && dz.numel() == dh.numel() &&
                  dh.numel() % 8 == 0 && p >= 0.0 && p < 1.0,
              "fc_act_bwd: bad sizes");
  pdt::fc_act_bwd_launch(dt, p16(dh, "dh"), p16(out, "out"), p16(dz, "dz"), dh.numel(), p, cur_stream());
  launched("fc_act_bwd_launch");
}

void nhwc_nchw16(const Tensor& src, Tensor& dst, int64_t N, int64_t HW, int64_t C, bool to_nchw) {
  const int dt = dt16(src, "src");
  TORCH_CHECK(dt16(dst, "dst") == dt && src.numel() == N * HW * C && dst.numel() == src.numel(), "nhwc_nchw16: bad sizes");
  pdt::nhwc_nchw16_launch(p16(src, "src"), p16(dst, "dst"), N, (int)HW, (int)C, to_nchw, cur_stream());
  launched("nhwc_nchw16_launch");
}

void bias_coef(const Tensor& bias, Tensor& coef, int64_t C) {
  TORCH_CHECK(bias.numel() >= C && coef.numel() >= 4 * C, "bias_coef: bad sizes");
  pdt::bias_coef_launch(pf(bias, "bias"), pf(coef, "coef"), (int)C, cur_stream());
  launched("bias_coef_launch");
}

// ... and apply pass writing dy = A*dz + B*y + C (bcoef from bn_bwd_finalize)
void stem_pool_bwd_apply(const Tensor& dp, const Tensor& idx, const Tensor& y, const Tensor& coef,
                         const Tensor& bcoef, Tensor& dy, int64_t N, int64_t H, int64_t W, int64_t C) {
  const int dt = dt16(dp, "dp");
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dt16(y, "y") == dt && dt16(dy, "dy") == dt && dp.numel() == N * OH * OW * C &&
                  y.numel() == N * H * W * C && dy.numel() == y.numel() && idx.numel() == dp.numel() &&
                  C % 8 == 0 && coef.numel() >= 2 * C && bcoef.numel() >= 3 * C,
              "stem_pool_bwd_apply: bad sizes");
  TORCH_CHECK(y.numel() < (int64_t(1) << 32), "stem_pool_bwd_apply: tensor exceeds 2^32 elements (32-bit indexing)");
  check_dev(idx, "idx");
  pdt::stem_pool_bwd_apply_launch(dt, p16(dp, "dp"), idx.data_ptr<uint8_t>(), p16(y, "y"), pf(coef, "coef"),
                                  pf(bcoef, "bcoef"), p16(dy, "dy"), N, H, W, C, cur_stream());
  launched("stem_pool_bwd_apply_launch");
}

void avgpool_fwd(const Tensor& x, Tensor& feat, int64_t N, int64_t HW, int64_t C, int64_t ldf) {
  const int dt = dt16(x, "x");
  TORCH_CHECK(x.numel() == N * HW * C && feat.numel() >= N * ldf && C % 8 == 0, "avgpool_fwd: bad sizes");
  pdt::avgpool_fwd_launch(dt, p16(x, "x"), p16(feat, "feat"), N, HW, C, ldf, cur_stream());
  launched("avgpool_fwd_launch");
}

void avgpool_bwd(const Tensor& dfeat, Tensor& g, int64_t N, int64_t HW, int64_t C, int64_t ldf) {
  const int dt = dt16(dfeat, "dfeat");
  TORCH_CHECK(g.numel() == N * HW * C && dfeat.numel() >= N * ldf && C % 8 == 0, "avgpool_bwd: bad sizes");
  pdt::avgpool_bwd_launch(dt, p16(dfeat, "dfeat"), p16(g, "g"), N, HW, C, ldf, cur_stream());
  launched("avgpool_bwd_launch");
}

// ------------------------------------------------------------------------------------------ loss
void xent(const Tensor& logits, int64_t ldl, const OptT& bias, const Tensor& target, int64_t B, int64_t ncls,
          const OptT& out_logits, const OptT& dlogits, const OptT& loss_scale, double grad_div, Tensor& row_loss,
          Tensor& row_correct) {
  const int dt = dt16(logits, "logits");
  check_dev(target, "target");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == B, "xent: target must be int64 [B]");
  TORCH_CHECK(logits.numel() >= B * ldl && ncls <= ldl, "xent: logits too small");
  if (out_logits.has_value()) TORCH_CHECK(out_logits->numel() == B * ncls, "xent: out_logits size");
  if (dlogits.has_value()) TORCH_CHECK(dlogits->numel() >= B * ldl, "xent: dlogits size");
  pdt::xent_launch(dt, p16(logits, "logits"), ldl, pfo(bias, "bias"), target.data_ptr<int64_t>(), B, ncls,
                   pfo(out_logits, "out_logits"), p16m(dlogits, "dlogits"), pfo(loss_scale, "loss_scale"),
                   (float)grad_div, pf(row_loss, "row_loss"), pf(row_correct, "row_correct"), cur_stream());
  launched("xent_launch");
}

void metrics(const Tensor& row_loss, const Tensor& row_correct, int64_t B, Tensor& out) {
  pdt::metrics_launch(pf(row_loss, "row_loss"), pf(row_correct, "row_correct"), B, pf(out, "out"), cur_stream());
  launched("metrics_launch");
}

void colsum(const Tensor& d, int64_t B, int64_t ld, int64_t ncols, Tensor& out, double scale) {
  const int dt = dt16(d, "d");
  TORCH_CHECK(d.numel() >= B * ld && out.numel() >= ncols, "colsum: bad sizes");
  pdt::colsum_launch(dt, p16(d, "d"), B, ld, ncols, pf(out, "out"), (float)scale, cur_stream());
  launched("colsum_launch");
}

// ----------------------------------------------------------------------------------------- optim
void nonfinite_check(const Tensor& g, Tensor& found) {
  pdt::nonfinite_check_launch(pf(g, "g"), g.numel(), pf(found, "found"), cur_stream());
  launched("nonfinite_check_launch");
}

void sgd(Tensor& p, const Tensor& g, Tensor& buf, const OptT& shadow, const OptT& wd_mask, double lr, double momentum,
         double wd, double gscale, const OptT& loss_scale, const OptT& found_inf, bool first) {
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && buf.numel() == n, "sgd: size mismatch");
  int dt = pdt::kBF16;
  if (shadow.has_value()) {
    dt = dt16(*shadow, "shadow");
    TORCH_CHECK(shadow->numel() == n, "sgd: shadow size mismatch");
  }
  if (wd_mask.has_value()) TORCH_CHECK(wd_mask->numel() == n, "sgd: wd_mask size mismatch");
  pdt::sgd_launch(dt, pf(p, "p"), pf(g, "g"), pf(buf, "buf"), p16m(shadow, "shadow"), pfo(wd_mask, "wd_mask"), n,
                  (float)lr, (float)momentum, (float)wd, (float)gscale, pfo(loss_scale, "loss_scale"),
                  pfo(found_inf, "found_inf"), first, cur_stream());
  launched("sgd_launch");
}

void cast16(const Tensor& p, Tensor& out) {
  TORCH_CHECK(p.numel() == out.numel(), "cast16: size mismatch");
  pdt::cast16_launch(dt16(out, "out"), pf(p, "p"), p16(out, "out"), p.numel(), cur_stream());
  launched("cast16_launch");
}

void amp_update(Tensor& scale, Tensor& tracker, Tensor& found_inf, double growth, double backoff, int64_t interval) {
  check_dev(tracker, "tracker");
  TORCH_CHECK(tracker.scalar_type() == at::kInt, "amp_update: tracker must be int32");
  pdt::amp_update_launch(pf(scale, "scale"), tracker.data_ptr<int>(), pf(found_inf, "found_inf"), (float)growth,
                         (float)backoff, (int)interval, cur_stream());
  launched("amp_update_launch");
}

void gather16(const Tensor& src, const Tensor& idx, Tensor& dst) {
  check_dev(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.numel() == dst.numel(), "gather16: idx must be int32 like dst");
  pdt::gather16_launch(p16(src, "src"), idx.data_ptr<int>(), p16(dst, "dst"), dst.numel(), cur_stream());
  launched("gather16_launch");
}

void im2col(const Tensor& x, Tensor& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
            int64_t stride, int64_t pad, int64_t ldk) {
  const int dt = dt16(out, "out");
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(x.numel() == N * C * H * W && out.numel() == N * OH * OW * ldk && ldk % 8 == 0 && ldk >= R * S * C,
              "im2col: bad sizes");
  pdt::im2col_launch(dt, pf(x, "x"), p16(out, "out"), N, C, H, W, R, S, stride, pad, ldk, cur_stream());
  launched("im2col_launch");
}

void stem_pack(const Tensor& x, Tensor& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t pad, int64_t Hp,
               int64_t Wp) {
  TORCH_CHECK(x.numel() == N * C * H * W && out.numel() == N * Hp * Wp * 4 && C <= 4 && Hp >= H + 2 * pad &&
                  Wp >= W + 2 * pad && N * Hp * Wp < (int64_t(1) << 31), "stem_pack: bad sizes");
  pdt::stem_pack_launch(dt16(out, "out"), pf(x, "x"), p16(out, "out"), N, C, H, W, pad, Hp, Wp, cur_stream());
  launched("stem_pack_launch");
}

// uint8 NCHW pixels -> normalised, zero-padded NHWC4 16-bit stem input (v = x * scale[c] + shift[c])
void stem_pack_u8(const Tensor& x, Tensor& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t pad, int64_t Hp,
                  int64_t Wp, const Tensor& scale, const Tensor& shift) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kByte, "stem_pack_u8: x must be uint8");
  TORCH_CHECK(x.numel() == N * C * H * W && out.numel() == N * Hp * Wp * 4 && C <= 4 && Hp >= H + 2 * pad &&
                  Wp >= W + 2 * pad && scale.numel() >= C && shift.numel() >= C && N * Hp * Wp < (int64_t(1) << 31),
              "stem_pack_u8: bad sizes");
  pdt::stem_pack_u8_launch(dt16(out, "out"), x.data_ptr<uint8_t>(), p16(out, "out"), N, C, H, W, pad, Hp, Wp,
                           pf(scale, "scale"), pf(shift, "shift"), cur_stream());
  launched("stem_pack_u8_launch");
}

void bw_probe(int64_t mode, const Tensor& x, const Tensor& y, Tensor& out, int64_t blocks) {
  TORCH_CHECK(x.numel() == y.numel() && out.numel() == x.numel() && x.numel() % 8 == 0, "bw_probe: sizes");
  pdt::bw_probe_launch((int)mode, p16(x, "x"), p16(y, "y"), p16(out, "out"), x.numel(), (int)blocks, cur_stream());
  launched("bw_probe_launch");
}

void gather32(const Tensor& src, const Tensor& idx, Tensor& dst) {
  check_dev(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.numel() == dst.numel(), "gather32: idx must be int32 like dst");
  pdt::gather32_launch(pf(src, "src"), idx.data_ptr<int>(), pf(dst, "dst"), dst.numel(), cur_stream());
  launched("gather32_launch");
}

// dst[idx[i]] = src[i]; the caller guarantees 0 <= idx < dst.numel() (checked where the index map is built)
void scatter32(const Tensor& src, const Tensor& idx, Tensor& dst) {
  check_dev(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.numel() == src.numel(), "scatter32: idx must be int32 like src");
  pdt::scatter32_launch(pf(src, "src"), idx.data_ptr<int>(), pf(dst, "dst"), src.numel(), cur_stream());
  launched("scatter32_launch");
}

// ------------------------------------------------------------------------------------------ fp32 path
const float* pfc(const OptT& t, const char* name) { return t.has_value() ? pf(*t, name) : nullptr; }

// forward conv over fp32 NHWC / KRSC (same geometry arguments as conv_fwd; stats -> fp64 slots)
void conv32_fwd(const Tensor& x, const Tensor& w, Tensor& y, const OptT& res, const OptT& stats, int64_t N, int64_t H,
                int64_t W, int64_t C, int64_t Kout, int64_t T, int64_t U, int64_t Pm, int64_t Qm, int64_t stride,
                int64_t pad, int64_t bm, int64_t bn) {
  TORCH_CHECK(x.numel() == N * H * W * C && w.numel() == Kout * T * U * C && y.numel() == N * Pm * Qm * Kout,
              "conv32_fwd: size mismatch");
  TORCH_CHECK(C % 32 == 0 && Kout % bn == 0, "conv32_fwd: C % 32 / Kout % bn must be 0");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && w.numel() < (int64_t(1) << 30) && N * Pm * Qm < (int64_t(1) << 31),
              "conv32_fwd: operands exceed 4 GiB (32-bit buffer offsets)");
  pdt::Conv32Args a{};
  a.x = pf(x, "x"); a.w = pf(w, "w"); a.y = pf(y, "y");
  if (res.has_value()) {
    TORCH_CHECK(res->numel() == y.numel(), "conv32_fwd: residual size");
    a.res = pf(*res, "res");
  }
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * Kout * 2, "conv32_fwd: stats buffer too small");
    a.stats = pd(*stats, "stats");
  }
  a.N = N; a.H = H; a.W = W; a.C = C; a.Kout = Kout; a.T = T; a.U = U; a.Pm = Pm; a.Qm = Qm;
  a.ist_h = stride; a.ist_w = stride; a.ioff_h = -pad; a.ioff_w = -pad; a.tstep_h = 1; a.tstep_w = 1;
  a.OH = Pm; a.OW = Qm; a.ost_h = 1; a.ost_w = 1; a.ooff_h = 0; a.ooff_w = 0;
  a.M = N * Pm * Qm;
  pdt::conv32_launch(a, (int)bm, (int)bn, cur_stream());
  launched("conv32_launch");
}

// backward-data over fp32 in ONE launch for every sub-pixel phase (phases as in conv_dgrad)
void conv32_dgrad(const Tensor& dy, const Tensor& wt, Tensor& dx, const OptT& res, int64_t N, int64_t P, int64_t Q,
                  int64_t K, int64_t C, int64_t H, int64_t W, int64_t stride,
                  const std::vector<std::vector<int64_t>>& phases, int64_t bm, int64_t bn, const OptT& bn_mref = {},
                  const OptT& bn_y1 = {}, const OptT& bn_coef = {}, const OptT& stats = {}, const OptT& bn_y2 = {},
                  const OptT& bn_coef2 = {}) {
  TORCH_CHECK(dy.numel() == N * P * Q * K && dx.numel() == N * H * W * C, "conv32_dgrad: size mismatch");
  TORCH_CHECK(K % 32 == 0 && C % bn == 0, "conv32_dgrad: K % 32 / C % bn must be 0");
  TORCH_CHECK(dy.numel() < (int64_t(1) << 30) && wt.numel() < (int64_t(1) << 30), "conv32_dgrad: operands too large");
  TORCH_CHECK(!phases.empty() && phases.size() <= 4, "conv32_dgrad: 1..4 phases");
  pdt::Conv32Args a{};
  a.x = pf(dy, "dy"); a.w = pf(wt, "wt"); a.y = pf(dx, "dx");
  if (res.has_value()) {
    TORCH_CHECK(res->numel() == dx.numel(), "conv32_dgrad: residual size");
    a.res = pf(*res, "res");
  }
  if (bn_y1.has_value()) {  // fused BN-backward reduce (Conv32Args::bnb); no mref: ReLU mask from y1 * scale + shift
    TORCH_CHECK(bn_coef.has_value() && stats.has_value(),
                "conv32_dgrad: the fused BN-backward reduce needs y1, coef and stats");
    const int64_t KO = bn_y2.has_value() ? 4 : 2;
    TORCH_CHECK((!bn_mref.has_value() || bn_mref->numel() == dx.numel()) && bn_y1->numel() == dx.numel() &&
                bn_coef->numel() >= 4 * C && stats->numel() >= pdt::kStatSlots * C * KO,
                "conv32_dgrad: fused BN-backward operand sizes");
    a.bnb = 1;
    TORCH_CHECK(bn_mref.has_value() || !bn_y2.has_value(), "conv32_dgrad: two BN branches need the mask reference");
    a.bn_mref = bn_mref.has_value() ? pf(*bn_mref, "bn_mref") : nullptr;
    a.bn_y1 = pf(*bn_y1, "bn_y1"); a.bn_coef = pf(*bn_coef, "bn_coef");
    a.stats = pd(*stats, "stats");
    if (bn_y2.has_value()) {
      TORCH_CHECK(bn_coef2.has_value() && bn_y2->numel() == dx.numel() && bn_coef2->numel() >= 4 * C,
                  "conv32_dgrad: second BN branch operands");
      a.bn_y2 = pf(*bn_y2, "bn_y2"); a.bn_coef2 = pf(*bn_coef2, "bn_coef2");
    }
  }
  a.N = N; a.H = P; a.W = Q; a.C = K; a.Kout = C;
  a.ist_h = 1; a.ist_w = 1; a.tstep_h = -1; a.tstep_w = -1;
  a.OH = H; a.OW = W; a.ost_h = stride; a.ost_w = stride;
  a.nphase = (int)phases.size();
  int64_t maxM = 0;
  for (size_t i = 0; i < phases.size(); ++i) {
    const auto& f = phases[i];
    TORCH_CHECK(f.size() == 7, "conv32_dgrad: phase = (ph, pw, T, U, ioff_h, ioff_w, woff)");
    const int64_t Pm = (H - f[0] + stride - 1) / stride, Qm = (W - f[1] + stride - 1) / stride;
    TORCH_CHECK(Pm > 0 && Qm > 0 && f[6] + C * f[2] * f[3] * K <= wt.numel(), "conv32_dgrad: bad phase");
    a.pooff_h[i] = (int)f[0]; a.pooff_w[i] = (int)f[1]; a.pT[i] = (int)f[2]; a.pU[i] = (int)f[3];
    a.pioff_h[i] = (int)f[4]; a.pioff_w[i] = (int)f[5]; a.pwoff[i] = f[6];
    a.pPm[i] = (int)Pm; a.pQm[i] = (int)Qm;
    maxM = std::max(maxM, N * Pm * Qm);
  }
  TORCH_CHECK(maxM < (int64_t(1) << 31), "conv32_dgrad: too many pixels");
  a.M = maxM;
  a.Pm = a.pPm[0]; a.Qm = a.pQm[0];
  pdt::conv32_launch(a, (int)bm, (int)bn, cur_stream());
  launched("conv32_launch");
}

void wgrad32(const Tensor& x, const Tensor& dy, Tensor& ws, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Kout,
             int64_t T, int64_t U, int64_t Pm, int64_t Qm, int64_t stride, int64_t pad, int64_t ldw, int64_t splits,
             int64_t pix_per_split, int64_t tile) {
  TORCH_CHECK(tile == 64 || tile == 128 || tile == 3, "wgrad32: tile must be 64, 128 or 3 (3x3 halo kernel)");
  const int64_t cb = tile == 3 ? 64 : tile;
  TORCH_CHECK(C % cb == 0 && Kout % cb == 0, "wgrad32: C and Kout must be multiples of the tile");
  TORCH_CHECK(x.numel() == N * H * W * C && dy.numel() == N * Pm * Qm * Kout, "wgrad32: size mismatch");
  TORCH_CHECK(x.numel() < (int64_t(1) << 30) && dy.numel() < (int64_t(1) << 30), "wgrad32: operands too large");
  TORCH_CHECK(ldw >= T * U * C && ws.numel() >= splits * Kout * ldw, "wgrad32: workspace too small");
  if (tile == 3) {  // halo kernel: splits over OUTPUT ROWS (N * Pm of them)
    TORCH_CHECK(pix_per_split > 0 && splits * pix_per_split >= N * Pm && T == 3 && U == 3 && stride == 1 && pad == 1 &&
                    Pm == H && Qm == W && Qm <= 62, "wgrad32: bad halo plan / geometry");
  } else {
    TORCH_CHECK(pix_per_split % 64 == 0 && splits * pix_per_split >= N * Pm * Qm, "wgrad32: bad split plan");
  }
  pdt::Wgrad32Args a{};
  a.tile = (int)tile;
  a.x = pf(x, "x"); a.dy = pf(dy, "dy"); a.ws = pf(ws, "ws");
  a.N = N; a.H = H; a.W = W; a.C = C; a.Kout = Kout; a.T = T; a.U = U; a.Pm = Pm; a.Qm = Qm;
  a.stride = stride; a.pad = pad; a.ldw = ldw; a.splits = splits; a.pix_per_split = pix_per_split;
  a.P = N * Pm * Qm;
  pdt::wgrad32_launch(a, cur_stream());
  launched("wgrad32_launch");
}

void bn_apply32(const Tensor& y, const Tensor& coef, const OptT& res, const OptT& rcoef, Tensor& out, int64_t C,
                int64_t resmode, bool relu) {
  TORCH_CHECK(C % 4 == 0 && y.numel() % C == 0 && out.numel() == y.numel(), "bn_apply32: bad sizes");
  if (resmode != 0) TORCH_CHECK(res.has_value() && res->numel() == y.numel(), "bn_apply32: residual");
  if (resmode == 2) TORCH_CHECK(rcoef.has_value(), "bn_apply32: residual coefficients");
  pdt::bn_apply32_launch(pf(y, "y"), pf(coef, "coef"), pfc(res, "res"), pfc(rcoef, "rcoef"), pf(out, "out"), y.numel(),
                         C, (int)resmode, relu, cur_stream());
  launched("bn_apply32_launch");
}

int64_t bn_bwd_reduce32_blocks(int64_t rows, int64_t C) { return pdt::bn_bwd_reduce32_blocks(rows, (int)C); }

void bn_bwd_reduce32(const Tensor& g, const OptT& mref, const Tensor& y1, const Tensor& coef1, const OptT& y2,
                     const OptT& coef2, Tensor& slots, int64_t blocks, int64_t rows, int64_t C) {
  TORCH_CHECK(C % 4 == 0 && C <= 2048 && g.numel() == rows * C && y1.numel() == rows * C, "bn_bwd_reduce32: sizes");
  if (mref.has_value()) TORCH_CHECK(mref->numel() == g.numel(), "bn_bwd_reduce32: mask reference size");
  const int K = y2.has_value() ? 4 : 2;
  TORCH_CHECK(slots.numel() >= pdt::kStatSlots * C * K, "bn_bwd_reduce32: slots too small");
  pdt::bn_bwd_reduce32_launch(pf(g, "g"), pfc(mref, "mref"), pf(y1, "y1"), pf(coef1, "coef1"), pfc(y2, "y2"),
                              pfc(coef2, "coef2"), pd(slots, "slots"), (int)blocks, rows, (int)C, cur_stream());
  launched("bn_bwd_reduce32_launch");
}

void bn_bwd_apply32(const Tensor& g, const OptT& mref, const Tensor& y1, const Tensor& b1, Tensor& dy1, const OptT& y2,
                    const OptT& b2, const OptT& dy2, const OptT& dz, int64_t C) {
  TORCH_CHECK(C % 4 == 0 && g.numel() % C == 0 && dy1.numel() == g.numel(), "bn_bwd_apply32: bad sizes");
  pdt::bn_bwd_apply32_launch(pf(g, "g"), pfc(mref, "mref"), pf(y1, "y1"), pf(b1, "b1"), pf(dy1, "dy1"), pfc(y2, "y2"),
                             pfc(b2, "b2"), dy2.has_value() ? pf(*dy2, "dy2") : nullptr,
                             dz.has_value() ? pf(*dz, "dz") : nullptr, g.numel(), C, cur_stream());
  launched("bn_bwd_apply32_launch");
}

void bn_relu_maxpool32(const Tensor& y, const Tensor& coef, Tensor& out, Tensor& idx, int64_t N, int64_t H, int64_t W,
                       int64_t C) {
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(y.numel() == N * H * W * C && out.numel() == N * OH * OW * C && idx.numel() == out.numel() && C % 4 == 0,
              "bn_relu_maxpool32: bad sizes");
  check_dev(idx, "idx");
  pdt::bn_relu_maxpool32_launch(pf(y, "y"), pf(coef, "coef"), pf(out, "out"), idx.data_ptr<uint8_t>(), N, H, W, C,
                                cur_stream());
  launched("bn_relu_maxpool32_launch");
}

// the stem's backward tail without the dz tensor: fused max-pool backward + ReLU mask + BN-backward reduce / apply
void stem_pool_bwd_reduce32(const Tensor& dp, const Tensor& idx, const Tensor& y, const Tensor& coef, Tensor& slots,
                            int64_t blocks, int64_t N, int64_t H, int64_t W, int64_t C) {
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dp.numel() == N * OH * OW * C && y.numel() == N * H * W * C && idx.numel() == dp.numel() && C % 4 == 0 &&
                  C / 4 <= 256 && 256 % (C / 4) == 0 && coef.numel() >= 4 * C && slots.numel() >= pdt::kStatSlots * C * 2 &&
                  N * H * W < (int64_t(1) << 31),
              "stem_pool_bwd_reduce32: bad sizes");
  check_dev(idx, "idx");
  pdt::stem_pool_bwd_reduce32_launch(pf(dp, "dp"), idx.data_ptr<uint8_t>(), pf(y, "y"), pf(coef, "coef"),
                                     pd(slots, "slots"), (int)blocks, N, H, W, C, cur_stream());
  launched("stem_pool_bwd_reduce32_launch");
}

void stem_pool_bwd_reduce_out32(const Tensor& dp, const Tensor& out, const Tensor& coef, Tensor& slots, int64_t blocks,
                                int64_t C) {
  TORCH_CHECK(dp.numel() == out.numel() && dp.numel() % C == 0 && C % 4 == 0 && C / 4 <= 256 && 256 % (C / 4) == 0 &&
                  coef.numel() >= 4 * C && slots.numel() >= pdt::kStatSlots * C * 2 && blocks >= 1,
              "stem_pool_bwd_reduce_out32: bad sizes");
  pdt::stem_pool_bwd_reduce_out32_launch(pf(dp, "dp"), pf(out, "out"), pf(coef, "coef"), pd(slots, "slots"),
                                         (int)blocks, dp.numel() / C, (int)C, cur_stream());
  launched("stem_pool_bwd_reduce_out32_launch");
}

void stem_pool_bwd_apply32(const Tensor& dp, const Tensor& idx, const Tensor& y, const Tensor& coef, const Tensor& b,
                           Tensor& dy, int64_t N, int64_t H, int64_t W, int64_t C) {
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dp.numel() == N * OH * OW * C && y.numel() == N * H * W * C && dy.numel() == y.numel() &&
                  idx.numel() == dp.numel() && C % 4 == 0 && coef.numel() >= 4 * C && b.numel() >= 3 * C &&
                  N * H * W < (int64_t(1) << 31),
              "stem_pool_bwd_apply32: bad sizes");
  check_dev(idx, "idx");
  pdt::stem_pool_bwd_apply32_launch(pf(dp, "dp"), idx.data_ptr<uint8_t>(), pf(y, "y"), pf(coef, "coef"), pf(b, "b"),
                                    pf(dy, "dy"), N, H, W, C, cur_stream());
  launched("stem_pool_bwd_apply32_launch");
}

void maxpool_bwd_relu32(const Tensor& dp, const Tensor& idx, const Tensor& y, const Tensor& coef, Tensor& dz, int64_t N,
                        int64_t H, int64_t W, int64_t C) {
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dp.numel() == N * OH * OW * C && y.numel() == N * H * W * C && dz.numel() == y.numel() &&
                  idx.numel() == dp.numel() && C % 4 == 0,
              "maxpool_bwd_relu32: bad sizes");
  check_dev(idx, "idx");
  pdt::maxpool_bwd_relu32_launch(pf(dp, "dp"), idx.data_ptr<uint8_t>(), pf(y, "y"), pf(coef, "coef"), pf(dz, "dz"), N, H,
                                 W, C, cur_stream());
  launched("maxpool_bwd_relu32_launch");
}

void avgpool32_fwd(const Tensor& x, Tensor& feat, int64_t N, int64_t HW, int64_t C, int64_t ldf) {
  TORCH_CHECK(x.numel() == N * HW * C && feat.numel() >= N * ldf, "avgpool32_fwd: bad sizes");
  pdt::avgpool32_fwd_launch(pf(x, "x"), pf(feat, "feat"), N, HW, C, ldf, cur_stream());
  launched("avgpool32_fwd_launch");
}

void avgpool32_bwd(const Tensor& dfeat, Tensor& g, int64_t N, int64_t HW, int64_t C, int64_t ldf) {
  TORCH_CHECK(g.numel() == N * HW * C && dfeat.numel() >= N * ldf, "avgpool32_bwd: bad sizes");
  pdt::avgpool32_bwd_launch(pf(dfeat, "dfeat"), pf(g, "g"), N, HW, C, ldf, cur_stream());
  launched("avgpool32_bwd_launch");
}

void xent32(const Tensor& logits, int64_t ldl, const OptT& bias, const Tensor& target, int64_t B, int64_t ncls,
            const OptT& out_logits, const OptT& dlogits, const OptT& loss_scale, double grad_div, Tensor& row_loss,
            Tensor& row_correct) {
  check_dev(target, "target");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == B, "xent32: target must be int64 [B]");
  TORCH_CHECK(logits.numel() >= B * ldl && ncls <= ldl, "xent32: logits too small");
  if (out_logits.has_value()) TORCH_CHECK(out_logits->numel() == B * ncls, "xent32: out_logits size");
  if (dlogits.has_value()) TORCH_CHECK(dlogits->numel() >= B * ldl, "xent32: dlogits size");
  pdt::xent32_launch(pf(logits, "logits"), ldl, pfc(bias, "bias"), target.data_ptr<int64_t>(), B, ncls,
                     out_logits.has_value() ? pf(*out_logits, "out_logits") : nullptr,
                     dlogits.has_value() ? pf(*dlogits, "dlogits") : nullptr, pfc(loss_scale, "loss_scale"),
                     (float)grad_div, pf(row_loss, "row_loss"), pf(row_correct, "row_correct"), cur_stream());
  launched("xent32_launch");
}

void colsum32(const Tensor& d, int64_t B, int64_t ld, int64_t ncols, Tensor& out, double scale) {
  TORCH_CHECK(d.numel() >= B * ld && out.numel() >= ncols, "colsum32: bad sizes");
  pdt::colsum32_launch(pf(d, "d"), B, ld, ncols, pf(out, "out"), (float)scale, cur_stream());
  launched("colsum32_launch");
}

// window-mode fp32 stem (conv32 over the zero-padded NHWC4 image, K = R kernel rows x 32: 8 pixels x 4 channels)
void stem_pack32(const Tensor& x, Tensor& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t pad, int64_t Hp,
                 int64_t Wp) {
  TORCH_CHECK(C <= 3 && x.numel() >= N * C * H * W && out.numel() == N * Hp * Wp * 4 && Hp >= H + 2 * pad &&
              Wp >= W + 2 * pad, "stem_pack32: sizes");
  pdt::stem_pack32_launch(pf(x, "x"), pf(out, "out"), N, C, H, W, pad, Hp, Wp, cur_stream());
  launched("stem_pack32_launch");
}

void conv32_stem_fwd(const Tensor& xp, const Tensor& w, Tensor& y, const OptT& stats, int64_t N, int64_t Hp, int64_t Wp,
                     int64_t R, int64_t P, int64_t Q, int64_t stride, int64_t Kout, int64_t bm, int64_t bn) {
  TORCH_CHECK(xp.numel() == N * Hp * Wp * 4 && w.numel() == Kout * R * 32 && y.numel() == N * P * Q * Kout,
              "conv32_stem_fwd: size mismatch");
  TORCH_CHECK((P - 1) * stride + R <= Hp && (Q - 1) * stride + 8 <= Wp && Kout % bn == 0,
              "conv32_stem_fwd: the padded image must hold every 8-pixel window");
  TORCH_CHECK(xp.numel() < (int64_t(1) << 30) && N * P * Q < (int64_t(1) << 31), "conv32_stem_fwd: operands too large");
  pdt::Conv32Args a{};
  a.x = pf(xp, "xp"); a.w = pf(w, "w"); a.y = pf(y, "y");
  if (stats.has_value()) {
    TORCH_CHECK(stats->numel() >= pdt::kStatSlots * Kout * 2, "conv32_stem_fwd: stats buffer too small");
    a.stats = pd(*stats, "stats");
  }
  a.N = N; a.H = Hp; a.W = Wp; a.C = 32; a.cs = 4; a.Kout = Kout; a.T = R; a.U = 1; a.Pm = P; a.Qm = Q;
  a.ist_h = stride; a.ist_w = stride; a.ioff_h = 0; a.ioff_w = 0; a.tstep_h = 1; a.tstep_w = 0;
  a.OH = P; a.OW = Q; a.ost_h = 1; a.ost_w = 1; a.ooff_h = 0; a.ooff_w = 0;
  a.M = N * P * Q;
  pdt::conv32_launch(a, (int)bm, (int)bn, cur_stream());
  launched("conv32_launch");
}

// fp32 stem weight gradient in window-pair mode over the zero-padded NHWC4 image (no im2col): "tap" t = kernel rows
// (2t, 2t+1), 64 columns = 8 pixels x 4 channels of each; ws[split][Kout][npairs * 64]
void wgrad32_stem(const Tensor& xp, const Tensor& dy, Tensor& ws, int64_t N, int64_t Hp, int64_t Wp, int64_t npairs,
                  int64_t Kout, int64_t P, int64_t Q, int64_t stride, int64_t splits, int64_t pix_per_split,
                  int64_t all_pairs = 0) {
  TORCH_CHECK(xp.numel() == N * Hp * Wp * 4 && dy.numel() == N * P * Q * Kout && Kout % 64 == 0, "wgrad32_stem: sizes");
  TORCH_CHECK((P - 1) * stride + 2 * npairs <= Hp && (Q - 1) * stride + 8 <= Wp, "wgrad32_stem: padded image too small");
  TORCH_CHECK(ws.numel() >= splits * Kout * npairs * 64 && pix_per_split % 64 == 0 && splits * pix_per_split >= N * P * Q,
              "wgrad32_stem: bad workspace / split plan");
  TORCH_CHECK(xp.numel() < (int64_t(1) << 30) && dy.numel() < (int64_t(1) << 30), "wgrad32_stem: operands too large");
  pdt::Wgrad32Args a{};
  a.tile = 64;
  a.x = pf(xp, "xp"); a.dy = pf(dy, "dy"); a.ws = pf(ws, "ws");
  a.N = N; a.H = Hp; a.W = Wp; a.C = 64; a.Kout = Kout; a.T = npairs; a.U = 1; a.Pm = P; a.Qm = Q;
  a.stride = stride; a.pad = 0; a.ldw = npairs * 64; a.splits = splits; a.pix_per_split = pix_per_split;
  a.P = N * P * Q;
  a.cs = 4; a.pair_skip = Wp * 4 - 32; a.tstep = 2;  // chunks 8..15 = the NEXT row's first 32 elements
  if (all_pairs) {  // wgrad32_stem4_kernel: one block per split covers every pair (needs 4 pairs)
    TORCH_CHECK(npairs == 4, "wgrad32_stem: all_pairs needs 4 kernel-row pairs");
    a.tile = 4;
  }
  pdt::wgrad32_launch(a, cur_stream());
  launched("wgrad32_launch");
}

// wgrad32_stem (4 pairs, all per block) with dY computed in the kernel from the stem's max-pool backward, ReLU mask and
// BN-backward apply (dp / idx: pooled gradient and argmax, y0: conv output, coef: forward scale | shift, bcoef: A | B |
// C): stem_pool_bwd_apply32 + wgrad32_stem without the dY tensor
void wgrad32_stem_fused(const Tensor& xp, const Tensor& dp, const Tensor& idx, const Tensor& y0, const Tensor& coef,
                        const Tensor& bcoef, Tensor& ws, int64_t N, int64_t Hp, int64_t Wp, int64_t P, int64_t Q,
                        int64_t stride, int64_t splits, int64_t pix_per_split) {
  const int64_t OH = (P - 1) / 2 + 1, OW = (Q - 1) / 2 + 1;  // 3x3/2 pad-1 max-pool output
  TORCH_CHECK(xp.numel() == N * Hp * Wp * 4 && y0.numel() == N * P * Q * 64 && dp.numel() == N * OH * OW * 64 &&
                  idx.numel() == dp.numel() && idx.scalar_type() == at::kByte && coef.numel() >= 128 &&
                  bcoef.numel() >= 192, "wgrad32_stem_fused: sizes");
  TORCH_CHECK((P - 1) * stride + 8 <= Hp && (Q - 1) * stride + 8 <= Wp, "wgrad32_stem_fused: padded image too small");
  TORCH_CHECK(ws.numel() >= splits * 64 * 256 && pix_per_split % 64 == 0 && splits * pix_per_split >= N * P * Q,
              "wgrad32_stem_fused: bad workspace / split plan");
  TORCH_CHECK(xp.numel() < (int64_t(1) << 30) && y0.numel() < (int64_t(1) << 31), "wgrad32_stem_fused: operands too large");
  check_dev(idx, "idx");
  pdt::Wgrad32Args a{};
  a.tile = 4;
  a.x = pf(xp, "xp"); a.dy = nullptr; a.ws = pf(ws, "ws");
  a.N = N; a.H = Hp; a.W = Wp; a.C = 64; a.Kout = 64; a.T = 4; a.U = 1; a.Pm = P; a.Qm = Q;
  a.stride = stride; a.pad = 0; a.ldw = 256; a.splits = splits; a.pix_per_split = pix_per_split;
  a.P = N * P * Q;
  a.cs = 4; a.pair_skip = Wp * 4 - 32; a.tstep = 2;
  a.f_dp = pf(dp, "dp"); a.f_idx = idx.data_ptr<uint8_t>(); a.f_y = pf(y0, "y0"); a.f_coef = pf(coef, "coef");
  a.f_bcoef = pf(bcoef, "bcoef"); a.f_OH = (int)OH; a.f_OW = (int)OW;
  pdt::wgrad32_launch(a, cur_stream());
  launched("wgrad32_launch");
}

void im2col32(const Tensor& x, Tensor& out, int64_t N, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
              int64_t stride, int64_t pad, int64_t ldk) {
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(x.numel() >= N * C * H * W && out.numel() == N * OH * OW * ldk && ldk >= R * S * C, "im2col32: sizes");
  pdt::im2col32_launch(pf(x, "x"), pf(out, "out"), N, C, H, W, R, S, stride, pad, ldk, cur_stream());
  launched("im2col32_launch");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  pdt_comm::register_comm(m);
  pdt_store::register_store(m);
  pdt_dp::register_dp(m);
  m.doc() = "gfx950 (MI355X) HIP kernels of pytorch_distributed_template_amd";
  m.def("dispatch_counts", []() {
    std::map<std::string, long long> out;
    auto& r = pdt::counters();
    std::lock_guard<std::mutex> lk(r.mu);
    for (auto& e : r.entries) out[e.first] = __atomic_load_n(e.second.get(), __ATOMIC_RELAXED);
    return out;
  });
  m.def("reset_dispatch_counts", []() {
    auto& r = pdt::counters();
    std::lock_guard<std::mutex> lk(r.mu);
    for (auto& e : r.entries) __atomic_store_n(e.second.get(), 0LL, __ATOMIC_RELAXED);
  });
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_m_tiles", &conv_m_tiles);
  m.def("conv_dgrad", &conv_dgrad);
  m.def("conv_dgrad_bn", &conv_dgrad_impl);
  m.def("conv_wgrad_plan", &conv_wgrad_plan);
  m.def("conv1x1_c64_supported", &conv1x1_c64_supported);
  m.def("conv1x1_c64", &conv1x1_c64, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stats"), py::arg("M"),
        py::arg("pre") = py::none());
  m.def("conv1x1_c64_mode", [](int64_t set) { return (int64_t)pdt::conv1x1_c64_mode((int)set); });
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("ws"), py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("C"), py::arg("Kout"), py::arg("T"), py::arg("U"), py::arg("Pm"), py::arg("Qm"), py::arg("stride_h"),
        py::arg("stride_w"), py::arg("pad_h"), py::arg("pad_w"), py::arg("dil_h"), py::arg("dil_w"), py::arg("ldw"),
        py::arg("splits"), py::arg("pix_per_split"), py::arg("cs"), py::arg("win"), py::arg("pre") = py::none());
  m.def("conv_wgrad_stem_fused", &conv_wgrad_stem_fused);
  m.def("gconv_fwd", &gconv_fwd);
  m.def("gconv_dgrad", &gconv_dgrad, py::arg("dy"), py::arg("wt"), py::arg("dx"), py::arg("N"), py::arg("P"),
        py::arg("Q"), py::arg("width"), py::arg("H"), py::arg("W"), py::arg("stride"), py::arg("phases"), py::arg("j"),
        py::arg("bm"), py::arg("bn"), py::arg("bn_y1") = py::none(), py::arg("bn_coef1") = py::none(),
        py::arg("bn_slots") = py::none());
  m.def("gconv_wgrad", &gconv_wgrad);
  m.def("gconv_slice", []() { return kGSlice; });
  m.def("gconv_wgrad_l1", &gconv_wgrad_l1);
  m.def("wgrad_reduce", &wgrad_reduce);
  m.def("wgrad_blocks_3x3c64", &wgrad_blocks_3x3c64);
  m.def("wgrad_3x3c64_supported", &wgrad_3x3c64_supported);
  m.def("conv_wgrad_3x3c64", &conv_wgrad_3x3c64, py::arg("x"), py::arg("dy"), py::arg("ws"), py::arg("N"), py::arg("H"),
        py::arg("W"), py::arg("pre_coef") = py::none());
  m.def("conv_fwd_pre", &conv_fwd_pre);
  m.def("conv1x1x", &conv1x1x);
  m.def("conv1x1x_supported", &conv1x1x_supported);
  m.def("conv_dgrad_persistent", &conv_dgrad_persistent);
  m.def("conv1x1x_mode", &conv1x1x_mode);
  m.def("conv1x1x_l1_mode", &conv1x1x_l1_mode);
  m.def("conv_fwd_pre_supported", &conv_fwd_pre_supported);
  m.def("bn_slot_sum", &bn_slot_sum);
  m.def("stat_slots", &stat_slots);
  m.def("conv_l1_set_pp", &pdt::conv_l1_set_pp, py::arg("mode"),
        "layer1 kernel choice: 1 = 8-wave ping-pong, 0 = 4-wave, -1 = PDT_CONV_L1_PP (default); returns the previous");
  m.def("conv32_set_halo", &pdt::conv32_set_halo, py::arg("on"),
        "fp32 3x3/s1 64-channel convolutions: 1 = halo kernel (default), 0 = per-tap "
        "restaging kernel; returns the previous setting");
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_finalize_slots", &bn_finalize_slots);
  m.def("bn_bwd_finalize_slots", &bn_bwd_finalize_slots);
  m.def("bn_eval_coef", &bn_eval_coef);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd_reduce_blocks", &bn_bwd_reduce_blocks);
  m.def("bn_bwd_reduce", &bn_bwd_reduce);
  m.def("bn_bwd_finalize", &bn_bwd_finalize);
  m.def("bn_bwd_apply", &bn_bwd_apply);
  m.def("bn_relu_maxpool", &bn_relu_maxpool, py::arg("y"), py::arg("coef"), py::arg("out"), py::arg("idx"),
        py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("pad") = 1);
  m.def("maxpool_bwd_relu", &maxpool_bwd_relu, py::arg("dp"), py::arg("idx"), py::arg("y"), py::arg("coef"),
        py::arg("dz"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("pad") = 1);
  m.def("stem_fwd", &stem_fwd);
  m.def("stem_fwd_supported", [](int64_t Hp, int64_t Wp, int64_t P, int64_t Q) {
    return pdt::stem_fwd_supported((int)Hp, (int)Wp, (int)P, (int)Q);
  });
  m.def("stem_pool_bwd_reduce", &stem_pool_bwd_reduce);
  m.def("stem_pool_bwd_reduce_out", &stem_pool_bwd_reduce_out);
  m.def("stem_pool_bwd_apply", &stem_pool_bwd_apply);
  m.def("bn_relu_maxpool2", &bn_relu_maxpool2, py::arg("y"), py::arg("coef"), py::arg("out"), py::arg("idx"), py::arg("N"),
        py::arg("H"), py::arg("W"), py::arg("C"));
  m.def("maxpool2_bwd", &maxpool2_bwd);
  m.def("pooled_bwd_reduce", &pooled_bwd_reduce);
  m.def("fc_act_fwd", &fc_act_fwd);
  m.def("fc_act_bwd", &fc_act_bwd);
  m.def("nhwc_nchw16", &nhwc_nchw16);
  m.def("bias_coef", &bias_coef);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("xent", &xent);
  m.def("metrics", &metrics);
  m.def("colsum", &colsum);
  m.def("nonfinite_check", &nonfinite_check);
  m.def("sgd", &sgd);
  m.def("cast16", &cast16);
  m.def("amp_update", &amp_update);
  m.def("gather16", &gather16);
  m.def("im2col", &im2col);
  m.def("stem_pack", &stem_pack);
  m.def("stem_pack_u8", &stem_pack_u8);
  m.def("gather32", &gather32);
  m.def("scatter32", &scatter32);
  m.def("bw_probe", &bw_probe);
  m.def("conv32_fwd", &conv32_fwd);
  m.def("conv32_dgrad", &conv32_dgrad, py::arg("dy"), py::arg("wt"), py::arg("dx"), py::arg("res"), py::arg("N"),
        py::arg("P"), py::arg("Q"), py::arg("K"), py::arg("C"), py::arg("H"), py::arg("W"), py::arg("stride"),
        py::arg("phases"), py::arg("bm"), py::arg("bn"), py::arg("bn_mref") = py::none(), py::arg("bn_y1") = py::none(),
        py::arg("bn_coef") = py::none(), py::arg("stats") = py::none(), py::arg("bn_y2") = py::none(),
        py::arg("bn_coef2") = py::none());
  m.def("wgrad32", &wgrad32);
  m.def("bn_apply32", &bn_apply32);
  m.def("bn_bwd_reduce32_blocks", &bn_bwd_reduce32_blocks);
  m.def("bn_bwd_reduce32", &bn_bwd_reduce32);
  m.def("bn_bwd_apply32", &bn_bwd_apply32);
  m.def("bn_relu_maxpool32", &bn_relu_maxpool32);
  m.def("maxpool_bwd_relu32", &maxpool_bwd_relu32);
  m.def("stem_pool_bwd_reduce32", &stem_pool_bwd_reduce32);
  m.def("stem_pool_bwd_apply32", &stem_pool_bwd_apply32);
  m.def("stem_pool_bwd_reduce_out32", &stem_pool_bwd_reduce_out32);
  m.def("avgpool32_fwd", &avgpool32_fwd);
  m.def("avgpool32_bwd", &avgpool32_bwd);
  m.def("xent32", &xent32);
  m.def("colsum32", &colsum32);
  m.def("stem_pack32", &stem_pack32);
  m.def("conv32_stem_fwd", &conv32_stem_fwd);
  m.def("wgrad32_stem_fused", &wgrad32_stem_fused);
  m.def("wgrad32_stem", &wgrad32_stem, py::arg("xp"), py::arg("dy"), py::arg("ws"), py::arg("N"), py::arg("Hp"),
        py::arg("Wp"), py::arg("npairs"), py::arg("Kout"), py::arg("P"), py::arg("Q"), py::arg("stride"),
        py::arg("splits"), py::arg("pix_per_split"), py::arg("all_pairs") = 0);
  m.def("im2col32", &im2col32);
}
