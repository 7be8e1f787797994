// Shared definitions for the gfx950 (CDNA4 / MI355X) kernels of pytorch_distributed_template_amd.
//
// Activations are NHWC, 16-bit (bf16 or fp16) storage; accumulation and all statistics are fp32.
// Every kernel is written for wave64; block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dtypes.h"

#define PDT_DEVICE __device__ __forceinline__

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

namespace pdt {

// 16-bit element traits: storage is uint16_t, math is fp32.
template <int DT> struct E16;
template <> struct E16<kBF16> {
  typedef bf16x8_t vec8;
  static PDT_DEVICE float to_f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
  static PDT_DEVICE uint16_t from_f(float f) {
    __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN stays NaN
    return __builtin_bit_cast(uint16_t, b);
  }
  // two values rounded and packed (lo | hi << 16) by ONE v_cvt_pk_bf16_f32 (from_f twice + shift / or: 4 VALU)
  static PDT_DEVICE uint32_t pack2(float lo, float hi) {
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    typedef float f32x2_t __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
  }
  static PDT_DEVICE f32x4_t mfma16x16x32(vec8 a, vec8 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct E16<kF16> {
  typedef f16x8_t vec8;
  static PDT_DEVICE float to_f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
  static PDT_DEVICE uint16_t from_f(float f) {
    // round the fp32 value itself: the opaque asm keeps the compiler from fusing the fma that produced f into a
    // v_fma_mixlo_f16 (one rounding straight to f16) in some kernels and not in others -- two kernels rounding
    // the same fp32 expression (bn_apply vs the fused producer BN of conv_l1) must agree bit for bit
    asm("" : "+v"(f));
    return __builtin_bit_cast(uint16_t, (_Float16)f);
  }
  static PDT_DEVICE uint32_t pack2(float lo, float hi) { return (uint32_t)from_f(lo) | ((uint32_t)from_f(hi) << 16); }
  static PDT_DEVICE f32x4_t mfma16x16x32(vec8 a, vec8 b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};


// the 8 16-bit values of a packed 16-byte vector (element 2i in the low half of dword i)
PDT_DEVICE void unpack8(uint4 v, uint16_t (&o)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = (uint16_t)w[i];
    o[2 * i + 1] = (uint16_t)(w[i] >> 16);
  }
}

// Producer BatchNorm + ReLU applied to a 16-byte chunk (8 channels) of an activation tile already staged in LDS
// (the BN1 -> ReLU -> conv2 chain of a residual block without the materialised activation).
// Bit-identical to bn_apply: the same fma(y, scale, shift) in fp32 and the same rounding; ReLU is taken on the
// rounded 16-bit values (max as signed 16-bit integers against +0: every negative value, -0 included, has the
// sign bit), which equals rounding after the fp32 max.
typedef short pdt_s16x2 __attribute__((ext_vector_type(2)));
template <int DT>
PDT_DEVICE uint4 pre_act8(uint4 v, const float (&sc)[8], const float (&sh)[8]) {
  using E = E16<DT>;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = E::to_f((uint16_t)(w[e] & 0xffff)) * sc[2 * e] + sh[2 * e];
    const float hi = E::to_f((uint16_t)(w[e] >> 16)) * sc[2 * e + 1] + sh[2 * e + 1];
    const uint32_t pk = E::pack2(lo, hi);
    w[e] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(pdt_s16x2, pk), pdt_s16x2{0, 0}));
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// The same over a thread's share of a staged tile: chunk k at base + off[k] when ok[k].  All reads are issued
// before any write (the compiler cannot prove the chunks disjoint, so per-chunk read-modify-write would
// serialise one LDS round trip per chunk).
template <int DT, int NCH>
PDT_DEVICE void pre_act_chunks(char* base, const int (&off)[NCH], const bool (&ok)[NCH], const float (&sc)[8],
                               const float (&sh)[8]) {
  uint4 v[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) v[k] = *(const uint4*)(base + off[k]);
#pragma unroll
  for (int k = 0; k < NCH; ++k)
    if (ok[k]) *(uint4*)(base + off[k]) = pre_act8<DT>(v[k], sc, sh);
}

// 16-byte streaming (nontemporal) global load / store for the elementwise passes: the activations they
// touch are hundreds of MB and are not re-read from L2 before eviction (tools/bw_probe.py:
// 5.0 TB/s for grid-stride cached loops vs 6.2-6.5 TB/s for one-vector-per-thread streaming grids).
typedef uint32_t pdt_u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
PDT_DEVICE uint4 ld16(const void* p) {
  if constexpr (NT) {
    const pdt_u32x4 t = __builtin_nontemporal_load((const pdt_u32x4*)p);
    return make_uint4(t[0], t[1], t[2], t[3]);
  } else {
    return *(const uint4*)p;
  }
}
template <bool NT>
PDT_DEVICE void st16(void* p, uint4 v) {
  if constexpr (NT) {
    const pdt_u32x4 t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, (pdt_u32x4*)p);
  } else {
    *(uint4*)p = v;
  }
}

// Inclusive scan over each 16-lane DPP row (row_shr 1, 2, 4, 8 with zero fill): lane 15 of every row
// ends with the sum of the row's 16 values.  Pure VALU (no LDS permute traffic).
PDT_DEVICE float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

PDT_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

PDT_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Exact unsigned division by a runtime constant for dividends < 2^31: q = umulhi(x, mul) >> shift
// (mul = ceil(2^(32+s)/d), s = floor(log2 d)); powers of two use mul = 0 (plain shift).
struct FastDiv {
  uint32_t mul;
  uint32_t shift;
};

inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((2ull << s) <= d) ++s;
  if ((d & (d - 1)) == 0) return FastDiv{0u, s};
  const uint64_t m = ((1ull << (32 + s)) + d - 1) / d;
  return FastDiv{(uint32_t)m, s};
}

PDT_DEVICE uint32_t fdiv(uint32_t x, FastDiv f) {
  return f.mul ? (__umulhi(x, f.mul) >> f.shift) : (x >> f.shift);
}

// Raw buffer resource (stride 0): LDS-DMA through buffer_load ... lds.  A byte offset at or beyond
// num_records reads zeros in hardware, which is how padding / tails are zero-filled (kOOB).
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr uint32_t kOOB = 0x80000000u;

PDT_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

PDT_DEVICE void buf_lds16(__amdgpu_buffer_rsrc_t r, void* lds_dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_dst, 16, voff, 0, 0, 0);
}

// The same LDS-DMA issued through inline asm: identical instruction, but invisible to the compiler's
// waitcnt pass, which otherwise drains EVERY in-flight LDS-DMA (s_waitcnt vmcnt(0)) in front of any
// ds_read_b64_tr_b16 (the transposed-read builtins carry no memory operand, so they may alias any
// pending DMA) -- that silently serialises a "prefetch next stage, compute current stage" loop.
// Callers order these DMAs themselves: an explicit (counted) s_waitcnt vmcnt + barrier before the
// first read of a staged buffer.
PDT_DEVICE void buf_lds16_asm(__amdgpu_buffer_rsrc_t r, void* lds_dst, uint32_t voff) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(lds_void_t*)lds_dst;  // LDS byte address (wave-uniform)
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0v), "v"(voff), "s"(r)
               : "m0");
}

// Global loads through inline asm, for kernels that count their vector-memory operations themselves
// (mixed with buf_lds16_asm): the compiler neither waits for them nor knows they are in flight, so the
// caller MUST s_waitcnt before any use -- with the loaded values as "+v" operands of that wait asm, so
// the uses cannot be scheduled ahead of it.
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
PDT_DEVICE u32x4v gload16_asm(const void* p) {
  u32x4v v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}
PDT_DEVICE u32x2v gload8_asm(const void* p) {
  u32x2v v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}

// XCD-aware bijective remap of a 1-D block index: blocks b and b+8 share an XCD under the
// observed round-robin dispatch, so give each XCD a contiguous range of logical tiles
// (speed only, never correctness: any placement is valid).
PDT_DEVICE int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, local = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

}  // namespace pdt

#define PDT_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) pdt_hip_fail(#expr, _e, __FILE__, __LINE__);             \
  } while (0)

void pdt_hip_fail(const char* expr, hipError_t e, const char* file, int line);

// Stream-ordered device scratch from PyTorch's caching allocator (defined in bindings.cpp): the memory may
// be released right after the launches that use it were enqueued on ``s`` -- the allocator hands it out
// again only to later work on the same stream (and hipGraph capture draws it from the graph's pool).
namespace pdt {
void* scratch_alloc(size_t bytes, hipStream_t s);
void scratch_free(void* p);
struct Scratch {
  void* p;
  Scratch(size_t bytes, hipStream_t s) : p(bytes ? scratch_alloc(bytes, s) : nullptr) {}
  ~Scratch() {
    if (p) scratch_free(p);
  }
  Scratch(const Scratch&) = delete;
  Scratch& operator=(const Scratch&) = delete;
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};
}  // namespace pdt

// Host-side kernel-dispatch counters (defined in bindings.cpp, read by C.dispatch_counts()): tests assert
// which specialised kernel variant a shape actually ran.  One relaxed atomic increment per launch.
// The counter is bound to ``name`` at the site's first execution: one literal name per call site.
namespace pdt {
long long* dispatch_counter(const char* name);
}
#define PDT_COUNT(name)                                                             \
  do {                                                                             \
    static long long* _pdt_ctr = pdt::dispatch_counter(name);                      \
    __atomic_fetch_add(_pdt_ctr, 1LL, __ATOMIC_RELAXED);                           \
  } while (0)
