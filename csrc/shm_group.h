// Host shared-memory collective group: the transport the native communicator (csrc/comm.cpp) uses when RCCL
// cannot -- ranks sharing one GPU (RCCL refuses duplicate devices), or CPU-only processes (tests) -- so the
// C++ Communicator / Bucketer multi-rank logic runs anywhere, not only on a multi-GPU node.
//
// One POSIX shared-memory segment per group: a header (sense-reversing barrier, abort flag) and one data slot
// per rank.  Collectives work on HOST memory in slot-sized chunks:
//   all_reduce: every rank copies its chunk into its slot, barrier, every rank reduces slot 0..W-1 IN RANK ORDER
//               into its own buffer (so all ranks hold bit-identical results, and the result does not depend on
//               timing: deterministic), barrier (slots free for the next chunk);
//   broadcast:  root copies into its slot, barrier, the others copy out, barrier;
//   all_gather: every rank copies into its slot, barrier, every rank copies all slots out, barrier.
// Failure handling: a barrier that waits longer than ``timeout_s`` (a peer died or hangs) raises, and sets the
// segment's abort flag so every other rank's barrier raises too instead of spinning forever.
//
// Header-only and free of HIP / torch so csrc/tests/shm_stress.cpp can drive it under ASan/UBSan/TSan.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace pdt_shm {

enum class Dt : int { F32 = 0, F64 = 1, F16 = 2, BF16 = 3, I32 = 4, I64 = 5, U8 = 6 };
enum class Op : int { Sum = 0, Max = 1, Min = 2, Prod = 3 };

inline size_t dt_size(Dt d) {
  switch (d) {
    case Dt::F64: case Dt::I64: return 8;
    case Dt::F32: case Dt::I32: return 4;
    case Dt::F16: case Dt::BF16: return 2;
    case Dt::U8: return 1;
  }
  return 1;
}

// 16-bit float <-> float (round to nearest even), host side
inline float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float f16_to_f(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  uint32_t u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {  // subnormal
      float f = std::ldexp((float)m, -24);
      std::memcpy(&u, &f, 4);
      u |= s;
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e + 112u) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f_to_f16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  const uint16_t s = (uint16_t)((u >> 16) & 0x8000u);
  const uint32_t a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return s | 0x7e00u;        // NaN
  if (a >= 0x477ff000u) return s | 0x7c00u;       // overflow -> inf (incl. rounding up past 65504)
  if (a < 0x38800000u) {                          // subnormal / zero: round (a * 2^24) to an integer
    const float af = std::fabs(f) * 16777216.0f;
    return s | (uint16_t)std::nearbyint(af);
  }
  uint32_t r = a - 0x38000000u;                   // rebias exponent 127 -> 15
  r += 0xfffu + ((r >> 13) & 1u);
  return s | (uint16_t)(r >> 13);
}

struct alignas(64) Header {
  std::atomic<uint32_t> arrive;
  std::atomic<uint32_t> gen;
  std::atomic<uint32_t> aborted;
  uint32_t world;
  uint64_t slot_bytes;
  uint64_t magic;
};
static_assert(sizeof(Header) <= 256, "header fits its 256-byte reservation");
constexpr uint64_t kMagic = 0x5044545348474d31ull;  // "PDTSHGM1"
constexpr size_t kHeaderBytes = 256;

class ShmGroup {
 public:
  // rank 0 passes create=true (O_EXCL: a stale segment of the same name is an error); the others open it after
  // rank 0 published the name.  unlink() once every rank has mapped it (after the first barrier).
  ShmGroup(const std::string& name, int world, int rank, bool create, size_t slot_bytes, double timeout_s)
      : name_(name), world_(world), rank_(rank), timeout_s_(timeout_s) {
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("shm group: bad rank / world");
    if (name.empty() || name[0] != '/') throw std::invalid_argument("shm group: name must start with '/'");
    const size_t total = kHeaderBytes + (size_t)world * slot_bytes;
    const auto t_open = std::chrono::steady_clock::now();
    int fd = -1;
    for (;;) {  // the non-creating ranks may get here before rank 0 created / sized the segment: retry
      fd = create ? shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) {
        if (!create && errno == ENOENT && elapsed(t_open) < timeout_s_) {
          std::this_thread::sleep_for(std::chrono::milliseconds(2));
          continue;
        }
        throw std::runtime_error("shm group: shm_open(" + name + ") failed: " + std::strerror(errno));
      }
      if (create && ftruncate(fd, (off_t)total) != 0) {
        const int e = errno;
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error(std::string("shm group: ftruncate failed: ") + std::strerror(e));
      }
      struct stat st {};
      if (fstat(fd, &st) == 0 && (size_t)st.st_size >= total) break;
      close(fd);
      if (create || elapsed(t_open) >= timeout_s_)
        throw std::runtime_error("shm group: segment " + name + " has the wrong size");
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error(std::string("shm group: mmap failed: ") + std::strerror(errno));
    base_ = static_cast<uint8_t*>(p);
    bytes_ = total;
    hdr_ = reinterpret_cast<Header*>(base_);
    if (create) {
      new (&hdr_->arrive) std::atomic<uint32_t>(0);
      new (&hdr_->gen) std::atomic<uint32_t>(0);
      new (&hdr_->aborted) std::atomic<uint32_t>(0);
      hdr_->world = (uint32_t)world;
      hdr_->slot_bytes = slot_bytes;
      std::atomic_thread_fence(std::memory_order_release);
      reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic) {
        if (elapsed(t0) > timeout_s_) throw std::runtime_error("shm group: segment never initialised");
        std::this_thread::yield();
      }
      if (hdr_->world != (uint32_t)world || hdr_->slot_bytes != slot_bytes)
        throw std::runtime_error("shm group: world / slot size differ from the creating rank's");
    }
    slot_bytes_ = slot_bytes;
  }
  ~ShmGroup() {
    if (base_) munmap(base_, bytes_);
  }
  ShmGroup(const ShmGroup&) = delete;
  ShmGroup& operator=(const ShmGroup&) = delete;

  int world() const { return world_; }
  int rank() const { return rank_; }
  size_t slot_bytes() const { return slot_bytes_; }
  void unlink() { shm_unlink(name_.c_str()); }
  bool aborted() const { return hdr_->aborted.load(std::memory_order_acquire) != 0; }
  void abort() { hdr_->aborted.store(1, std::memory_order_release); }

  void barrier() {
    if (aborted()) throw std::runtime_error("shm group: a peer aborted the group");
    const uint32_t g = hdr_->gen.load(std::memory_order_acquire);
    if (hdr_->arrive.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)world_ - 1) {
      hdr_->arrive.store(0, std::memory_order_relaxed);
      hdr_->gen.fetch_add(1, std::memory_order_acq_rel);
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    while (hdr_->gen.load(std::memory_order_acquire) == g) {
      // an abort raised AFTER the last rank completed this barrier must not fail it: re-check the generation
      if (aborted() && hdr_->gen.load(std::memory_order_acquire) == g)
        throw std::runtime_error("shm group: a peer aborted the group");
      if (++spins > 1024) {
        if (timeout_s_ > 0 && elapsed(t0) > timeout_s_) {
          abort();
          throw std::runtime_error("shm group: rank " + std::to_string(rank_) + " waited more than " +
                                   std::to_string(timeout_s_) + " s in a barrier (peer dead or hung)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(spins > 65536 ? 200 : 5));
      }
    }
  }

  uint8_t* slot(int r) { return base_ + kHeaderBytes + (size_t)r * slot_bytes_; }

  // in place over HOST memory; every rank ends with the same bits
  void all_reduce(void* buf, int64_t n, Dt dt, Op op) {
    const size_t es = dt_size(dt), per = slot_bytes_ / es;
    uint8_t* p = static_cast<uint8_t*>(buf);
    for (int64_t off = 0; off < n; off += (int64_t)per) {
      const size_t cnt = (size_t)std::min<int64_t>((int64_t)per, n - off);
      std::memcpy(slot(rank_), p + off * es, cnt * es);
      barrier();
      reduce_slots(p + off * es, cnt, dt, op);
      barrier();
    }
  }
  void broadcast(void* buf, int64_t n, Dt dt, int root) {
    const size_t es = dt_size(dt), per = slot_bytes_ / es;
    uint8_t* p = static_cast<uint8_t*>(buf);
    for (int64_t off = 0; off < n; off += (int64_t)per) {
      const size_t cnt = (size_t)std::min<int64_t>((int64_t)per, n - off);
      if (rank_ == root) std::memcpy(slot(root), p + off * es, cnt * es);
      barrier();
      if (rank_ != root) std::memcpy(p + off * es, slot(root), cnt * es);
      barrier();
    }
  }
  // out holds world x n elements, rank-major
  void all_gather(const void* in, void* out, int64_t n, Dt dt) {
    const size_t es = dt_size(dt), per = slot_bytes_ / es;
    const uint8_t* pi = static_cast<const uint8_t*>(in);
    uint8_t* po = static_cast<uint8_t*>(out);
    for (int64_t off = 0; off < n; off += (int64_t)per) {
      const size_t cnt = (size_t)std::min<int64_t>((int64_t)per, n - off);
      std::memcpy(slot(rank_), pi + off * es, cnt * es);
      barrier();
      for (int r = 0; r < world_; ++r) std::memcpy(po + ((size_t)r * n + off) * es, slot(r), cnt * es);
      barrier();
    }
  }

 private:
  static double elapsed(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  template <typename T>
  static T apply(Op op, T a, T b) {
    switch (op) {
      case Op::Sum: return a + b;
      case Op::Max: return a > b ? a : b;
      case Op::Min: return a < b ? a : b;
      case Op::Prod: return a * b;
    }
    return a;
  }
  template <typename T>
  void reduce_typed(T* dst, size_t cnt, Op op) {
    const T* s0 = reinterpret_cast<const T*>(slot(0));
    for (size_t i = 0; i < cnt; ++i) {
      T acc = s0[i];
      for (int r = 1; r < world_; ++r) acc = apply(op, acc, reinterpret_cast<const T*>(slot(r))[i]);
      dst[i] = acc;
    }
  }
  template <float (*ToF)(uint16_t), uint16_t (*FromF)(float)>
  void reduce_16(uint16_t* dst, size_t cnt, Op op) {
    // accumulate in fp32, one rounding at the end (rank order, like the other types)
    for (size_t i = 0; i < cnt; ++i) {
      float acc = ToF(reinterpret_cast<const uint16_t*>(slot(0))[i]);
      for (int r = 1; r < world_; ++r) acc = apply(op, acc, ToF(reinterpret_cast<const uint16_t*>(slot(r))[i]));
      dst[i] = FromF(acc);
    }
  }
  void reduce_slots(uint8_t* dst, size_t cnt, Dt dt, Op op) {
    switch (dt) {
      case Dt::F32: reduce_typed(reinterpret_cast<float*>(dst), cnt, op); break;
      case Dt::F64: reduce_typed(reinterpret_cast<double*>(dst), cnt, op); break;
      case Dt::I32: reduce_typed(reinterpret_cast<int32_t*>(dst), cnt, op); break;
      case Dt::I64: reduce_typed(reinterpret_cast<int64_t*>(dst), cnt, op); break;
      case Dt::U8: reduce_typed(reinterpret_cast<uint8_t*>(dst), cnt, op); break;
      case Dt::BF16: reduce_16<bf16_to_f, f_to_bf16>(reinterpret_cast<uint16_t*>(dst), cnt, op); break;
      case Dt::F16: reduce_16<f16_to_f, f_to_f16>(reinterpret_cast<uint16_t*>(dst), cnt, op); break;
    }
  }

  std::string name_;
  int world_, rank_;
  double timeout_s_;
  uint8_t* base_ = nullptr;
  size_t bytes_ = 0;
  size_t slot_bytes_ = 0;
  Header* hdr_ = nullptr;
};

}  // namespace pdt_shm
