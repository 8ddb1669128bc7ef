// Shared-memory control block of the parameter-server data plane (one per PS task).
//
// The between-graph PS of the reference (run_mnist_distributed.py:107-116, TF gRPC RecvTensor)
// moves every gradient and variable through the PS process.  Here the tensors never touch the
// host: gradients are written by the worker straight into a mailbox slot in the PS task's memory
// (HBM through a hipIpc mapping, or a /dev/shm file on CPU) and variables are read back the same
// way.  What remains on the host is this tiny block of sequence words in a MAP_SHARED /dev/shm
// segment, with futex sleep/wake so neither side spins:
//
//   worker w:  post(w, step)   slot FREE -> FULL, ring the owner's doorbell
//   owner:     wait_any()      FULL -> TAKEN for every posted slot (sleeps on the doorbell)
//   owner:     done(w, reply)  TAKEN -> DONE, wake worker w (reply = the new global step)
//   worker w:  wait_done(w)    DONE -> FREE, returns the reply
//
// Asynchronous training replies as soon as the update is applied; synchronous training
// (SyncReplicasOptimizer) holds the DONE of every contributor until the aggregated step closes,
// which is TF's token-queue barrier.  stop() wakes everyone and makes every later wait fail, so a
// PS shutdown or a dead peer can never strand a waiter.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

namespace dtf {

enum SlotState : uint32_t { kFree = 0, kFull = 1, kTaken = 2, kDone = 3 };

struct alignas(64) CtlCell {
  std::atomic<uint32_t> state;
  uint32_t pad0;
  int64_t step;     // global step the posted gradient was computed at
  int64_t reply;    // owner's answer (new global step), valid once DONE
  std::atomic<uint64_t> posts;   // lifetime counters (stats / tests)
  char pad[64 - 4 - 4 - 8 - 8 - 8];
};

struct alignas(64) CtlHeader {
  uint64_t magic;
  uint32_t n_workers;
  uint32_t pad0;
  std::atomic<uint32_t> doorbell;   // futex word the owner sleeps on
  std::atomic<uint32_t> stop;
  std::atomic<int64_t> global_step; // published by the owner after every apply
  std::atomic<uint64_t> heartbeat;  // owner liveness counter (bumped while serving)
  char pad[64 - 8 - 4 - 4 - 4 - 4 - 8 - 8];
};

class ShmControl {
 public:
  // create=true: the owner makes (and later unlinks) the segment; false: attach to it.
  ShmControl(const std::string& name, bool create, int n_workers);
  ~ShmControl();
  ShmControl(const ShmControl&) = delete;
  ShmControl& operator=(const ShmControl&) = delete;

  int n_workers() const { return (int)hdr_->n_workers; }
  const std::string& name() const { return name_; }

  // worker side
  void post(int w, int64_t step);
  // returns false on timeout; throws if stopped.  *reply = owner's answer
  bool wait_done(int w, int64_t timeout_ms, int64_t* reply);

  // owner side: fills `out` with posted (worker, step) pairs, returns count; 0 on timeout,
  // -1 once stopped.
  int wait_any(int64_t timeout_ms, int* workers, int64_t* steps, int cap);
  void done(int w, int64_t reply);
  void set_global_step(int64_t s) { hdr_->global_step.store(s, std::memory_order_release); }
  int64_t global_step() const { return hdr_->global_step.load(std::memory_order_acquire); }
  void beat() { hdr_->heartbeat.fetch_add(1, std::memory_order_relaxed); }
  uint64_t heartbeat() const { return hdr_->heartbeat.load(std::memory_order_relaxed); }
  uint64_t posts(int w) const { return cells_[w].posts.load(std::memory_order_relaxed); }
  uint32_t state(int w) const { return cells_[w].state.load(std::memory_order_acquire); }

  void stop();
  bool stopped() const { return hdr_->stop.load(std::memory_order_acquire) != 0; }
  void unlink();

 private:
  void check(int w) const;
  std::string name_;
  bool owner_;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  CtlHeader* hdr_ = nullptr;
  CtlCell* cells_ = nullptr;
};

}  // namespace dtf
