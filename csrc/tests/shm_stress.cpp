// Host-side stress driver for the shared-memory collective group (csrc/shm_group.h), built by
// tests/test_native_comm_cpu.py with AddressSanitizer + UndefinedBehaviorSanitizer and, separately, with
// ThreadSanitizer.  Every rank is a thread with its OWN mapping of the segment (as separate processes have), and
// runs many rounds of all_reduce (sum / max over f32, f64, bf16, i64, with payloads larger than a slot so the
// chunk loop and its two barriers per chunk are exercised), broadcast and all_gather, checking every result
// against its closed form; then one rank aborts and the others' barrier must raise instead of hanging.
//   shm_stress <ranks> <rounds>      exit 0 on success, 1 on a wrong result
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../shm_group.h"

using pdt_shm::Dt;
using pdt_shm::Op;
using pdt_shm::ShmGroup;

int main(int argc, char** argv) {
  const int world = argc > 1 ? std::atoi(argv[1]) : 4;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 20;
  const std::string name = "/pdt_shm_stress_" + std::to_string(getpid());
  const size_t slot = 4096;  // small: a 3000-float payload spans 3 chunks
  std::atomic<int> errors{0};
  auto fail = [&](const char* what, int r) {
    std::fprintf(stderr, "FAIL rank %d: %s\n", r, what);
    errors.fetch_add(1);
  };
  std::unique_ptr<ShmGroup> g0 = std::make_unique<ShmGroup>(name, world, 0, true, slot, 30.0);
  std::vector<std::thread> ts;
  std::atomic<int> aborted_seen{0};
  for (int r = 0; r < world; ++r) {
    ts.emplace_back([&, r] {
      try {
        std::unique_ptr<ShmGroup> own;
        ShmGroup* g = g0.get();
        if (r > 0) {
          own = std::make_unique<ShmGroup>(name, world, r, false, slot, 30.0);
          g = own.get();
        }
        g->barrier();
        if (r == 0) g->unlink();
        for (int it = 0; it < rounds; ++it) {
          std::vector<float> f(3000);
          for (size_t i = 0; i < f.size(); ++i) f[i] = (float)(r + 1) * (float)((i + it) % 7);
          g->all_reduce(f.data(), (int64_t)f.size(), Dt::F32, Op::Sum);
          const float tri = (float)(world * (world + 1) / 2);
          for (size_t i = 0; i < f.size(); ++i)
            if (f[i] != tri * (float)((i + it) % 7)) { fail("f32 sum", r); break; }
          std::vector<double> d(700);
          for (size_t i = 0; i < d.size(); ++i) d[i] = (double)(r * 1000 + (int)i);
          g->all_reduce(d.data(), (int64_t)d.size(), Dt::F64, Op::Max);
          for (size_t i = 0; i < d.size(); ++i)
            if (d[i] != (double)((world - 1) * 1000 + (int)i)) { fail("f64 max", r); break; }
          std::vector<uint16_t> h(2500);
          for (size_t i = 0; i < h.size(); ++i) h[i] = pdt_shm::f_to_bf16((float)(r + 1));
          g->all_reduce(h.data(), (int64_t)h.size(), Dt::BF16, Op::Sum);
          for (size_t i = 0; i < h.size(); ++i)
            if (pdt_shm::bf16_to_f(h[i]) != (float)(world * (world + 1) / 2)) { fail("bf16 sum", r); break; }
          std::vector<int64_t> b(1100, r == it % world ? 77 + it : -1);
          g->broadcast(b.data(), (int64_t)b.size(), Dt::I64, it % world);
          for (int64_t v : b)
            if (v != 77 + it) { fail("broadcast", r); break; }
          std::vector<int32_t> in(600, r * 10 + it), out(600 * world, -1);
          g->all_gather(in.data(), out.data(), (int64_t)in.size(), Dt::I32);
          for (int q = 0; q < world; ++q)
            if (out[(size_t)q * 600] != q * 10 + it || out[(size_t)q * 600 + 599] != q * 10 + it) {
              fail("all_gather", r);
              break;
            }
        }
        g->barrier();
        // failure path: the last rank aborts the group; everyone else's next barrier must raise
        if (r == world - 1) {
          g->abort();
        } else {
          try {
            g->barrier();
            fail("barrier returned after a peer aborted", r);
          } catch (const std::runtime_error&) {
            aborted_seen.fetch_add(1);
          }
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: exception %s\n", r, e.what());
        errors.fetch_add(1);
      }
    });
  }
  for (auto& t : ts) t.join();
  if (aborted_seen.load() != world - 1) fail("not every rank saw the abort", -1);
  std::printf("shm_stress: %d ranks x %d rounds, %d errors\n", world, rounds, errors.load());
  return errors.load() ? 1 : 0;
}
