// InputHandoff — the race-free replacement of the reference's unsynchronised hand-over of the
// solved inputs between project::OdomCallback (writer: current_inputs_ = solved_trajectory(),
// inputs_idx_ = 0; src/project.cpp:190-191) and the DriveLoop thread (reader: GetNextInput(),
// inputs_idx_++; :210-217,227-234). The reference shares both members without a lock (it
// includes <mutex> but never uses it, include/f110-mpc/project.h:13): a DriveLoop increment can
// be lost or applied to the new vector, and a read can see a vector being reassigned. Here one
// mutex guards the pair: Publish swaps in a new solution and resets the index atomically, Take
// returns the input at the index and advances it in the same critical section. Header-only so
// the ThreadSanitizer test (host/tests/handoff_tsan.cpp) compiles it without the GPU library.
#pragma once
#include <cstdio>
#include <mutex>
#include <utility>
#include <vector>

#include "f110mpc/input.h"

class InputHandoff {
 public:
  // OdomCallback side (project.cpp:190-191): the new solution replaces the old one, index 0.
  void Publish(std::vector<Input> inputs) {
    std::lock_guard<std::mutex> lk(mu_);
    inputs_.swap(inputs);
    idx_ = 0;
    ++generation_;
  }
  // GetNextInput (project.cpp:207-215): the input at the index, Input(0.5, 0) when exhausted.
  Input Peek(bool* ran_out = nullptr) const {
    std::lock_guard<std::mutex> lk(mu_);
    return at_locked(ran_out);
  }
  // One DriveLoop iteration's read + inputs_idx_++ (project.cpp:227-234), atomically.
  // *generation (optional) tells which Publish the input came from, *index its position.
  Input Take(unsigned long long* generation = nullptr, unsigned* index = nullptr) {
    std::lock_guard<std::mutex> lk(mu_);
    bool ran_out = false;
    const Input in = at_locked(&ran_out);
    if (generation) *generation = generation_;
    if (index) *index = idx_;
    ++idx_;
    return in;
  }
  std::vector<Input> Snapshot() const {
    std::lock_guard<std::mutex> lk(mu_);
    return inputs_;
  }
  unsigned index() const {
    std::lock_guard<std::mutex> lk(mu_);
    return idx_;
  }

 private:
  Input at_locked(bool* ran_out) const {
    if (idx_ >= inputs_.size()) {
      if (ran_out) *ran_out = true;
      return Input(0.5, 0.0);  // project.cpp:212-216 ("ran out of QP soln")
    }
    if (ran_out) *ran_out = false;
    return inputs_[idx_];
  }
  mutable std::mutex mu_;
  std::vector<Input> inputs_;
  unsigned idx_ = 0;
  unsigned long long generation_ = 0;
};
