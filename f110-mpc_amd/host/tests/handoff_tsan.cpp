// handoff_tsan.cpp — ThreadSanitizer check of the OdomCallback -> DriveLoop input hand-over.
//
// One writer thread plays project::OdomCallback (a new solved trajectory every few hundred us,
// src/project.cpp:190-191) while two reader threads play DriveLoop (GetNextInput + inputs_idx_++,
// :224-234) as fast as they can. Built twice by tests/test_host_threads.py with
// -fsanitize=thread: as is (InputHandoff, one mutex) it must run clean and every input a reader
// takes must be element `index` of the publication it came from (or the Input(0.5, 0) fallback
// past the end); with -DHANDOFF_REFERENCE the same threads use the reference's unsynchronised
// pair (a std::vector<Input> and an unsigned index shared without a lock), and ThreadSanitizer
// must report the race. Host code only: no GPU, no libf110qp.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "f110mpc/input_handoff.h"

namespace {

std::vector<Input> solution(unsigned gen, int n) {  // MPC::solved_trajectory of publication gen
  std::vector<Input> v;
  for (int k = 0; k < n; k++) v.emplace_back(static_cast<double>(gen), 1e-3 * k);
  return v;
}

#ifdef HANDOFF_REFERENCE
// the reference's members (project.h:60-61) and accesses (project.cpp:190-191, 210-217, 234)
struct ReferenceHandoff {
  std::vector<Input> current_inputs_;
  unsigned int inputs_idx_ = 0;
  unsigned long long gen_ = 0;
  void Publish(std::vector<Input> v) { current_inputs_ = v; inputs_idx_ = 0; ++gen_; }
  Input Take(unsigned long long* g, unsigned* i) {
    *g = gen_;
    *i = inputs_idx_;
    Input in = inputs_idx_ >= current_inputs_.size() ? Input(0.5, 0.0) : current_inputs_[inputs_idx_];
    inputs_idx_++;
    return in;
  }
};
using Handoff = ReferenceHandoff;
#else
using Handoff = InputHandoff;
#endif

}  // namespace

int main() {
  Handoff h;
  const int N = 30, kPublications = 2000;
  std::atomic<bool> done{false};
  std::atomic<long> bad{0}, taken{0}, fallback{0};
  h.Publish(solution(1, N));
  auto reader = [&] {
    while (!done) {
      unsigned long long g = 0;
      unsigned i = 0;
      const Input in = h.Take(&g, &i);
      taken++;
      if (i >= static_cast<unsigned>(N)) {
        fallback++;
        if (in.v() != 0.5 || in.steer_ang() != 0.0) bad++;
      } else if (in.v() != static_cast<double>(g) || in.steer_ang() != 1e-3 * i) {
        bad++;
      }
    }
  };
  std::thread r1(reader), r2(reader);
  for (unsigned g = 2; g < kPublications; g++) {
    h.Publish(solution(g, N));
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  done = true;
  r1.join();
  r2.join();
  std::printf("{\"taken\": %ld, \"fallback\": %ld, \"inconsistent\": %ld}\n", taken.load(), fallback.load(), bad.load());
  return bad.load() == 0 ? 0 : 3;
}
