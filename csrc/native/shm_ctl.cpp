#include "shm_ctl.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace dtf {

namespace {
constexpr uint64_t kMagic = 0x4454465053435431ull;  // "DTFPSCT1"

// Shared (not FUTEX_PRIVATE) futex: the word lives in a MAP_SHARED segment mapped by several
// processes.
long futex_wait(std::atomic<uint32_t>* w, uint32_t expect, int64_t timeout_ms) {
  struct timespec ts;
  struct timespec* tp = nullptr;
  if (timeout_ms >= 0) {
    ts.tv_sec = timeout_ms / 1000;
    ts.tv_nsec = (timeout_ms % 1000) * 1000000L;
    tp = &ts;
  }
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expect, tp, nullptr, 0);
}

void futex_wake(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, 0x7fffffff, nullptr, nullptr, 0);
}

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string shm_path(const std::string& name) { return "/" + name; }
}  // namespace

ShmControl::ShmControl(const std::string& name, bool create, int n_workers)
    : name_(name), owner_(create) {
  if (name.empty() || name.find('/') != std::string::npos)
    throw std::invalid_argument("ShmControl: name must be non-empty without '/'");
  int fd;
  if (create) {
    if (n_workers <= 0 || n_workers > 4096) throw std::invalid_argument("ShmControl: n_workers");
    bytes_ = sizeof(CtlHeader) + sizeof(CtlCell) * (size_t)n_workers;
    fd = shm_open(shm_path(name).c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("ShmControl: shm_open(create) " + name + ": " + strerror(errno));
    if (ftruncate(fd, (off_t)bytes_) != 0) {
      int e = errno;
      close(fd);
      shm_unlink(shm_path(name).c_str());
      throw std::runtime_error(std::string("ShmControl: ftruncate: ") + strerror(e));
    }
  } else {
    fd = shm_open(shm_path(name).c_str(), O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("ShmControl: shm_open(attach) " + name + ": " + strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(CtlHeader)) {
      close(fd);
      throw std::runtime_error("ShmControl: segment too small: " + name);
    }
    bytes_ = (size_t)st.st_size;
  }
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    if (create) shm_unlink(shm_path(name).c_str());
    throw std::runtime_error(std::string("ShmControl: mmap: ") + strerror(errno));
  }
  hdr_ = static_cast<CtlHeader*>(base_);
  cells_ = reinterpret_cast<CtlCell*>(static_cast<char*>(base_) + sizeof(CtlHeader));
  if (create) {
    std::memset(base_, 0, bytes_);      // fresh segment: every slot FREE
    hdr_->n_workers = (uint32_t)n_workers;
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else {
    if (hdr_->magic != kMagic) {
      munmap(base_, bytes_);
      base_ = nullptr;
      throw std::runtime_error("ShmControl: bad magic in " + name);
    }
    if (n_workers > 0 && (uint32_t)n_workers != hdr_->n_workers) {
      munmap(base_, bytes_);
      base_ = nullptr;
      throw std::runtime_error("ShmControl: worker count mismatch in " + name);
    }
    if (sizeof(CtlHeader) + sizeof(CtlCell) * (size_t)hdr_->n_workers > bytes_) {
      munmap(base_, bytes_);
      base_ = nullptr;
      throw std::runtime_error("ShmControl: truncated segment " + name);
    }
  }
}

ShmControl::~ShmControl() {
  if (base_) munmap(base_, bytes_);
  if (owner_) shm_unlink(shm_path(name_).c_str());
}

void ShmControl::unlink() {
  if (owner_) {
    shm_unlink(shm_path(name_).c_str());
    owner_ = false;
  }
}

void ShmControl::check(int w) const {
  if (w < 0 || (uint32_t)w >= hdr_->n_workers) throw std::out_of_range("ShmControl: worker index");
}

void ShmControl::post(int w, int64_t step) {
  check(w);
  CtlCell& c = cells_[w];
  if (stopped()) throw std::runtime_error("ShmControl: parameter server stopped");
  uint32_t s = c.state.load(std::memory_order_acquire);
  if (s != kFree) throw std::logic_error("ShmControl: post on a busy slot (missing wait_done)");
  c.step = step;
  c.posts.fetch_add(1, std::memory_order_relaxed);
  c.state.store(kFull, std::memory_order_release);
  hdr_->doorbell.fetch_add(1, std::memory_order_acq_rel);
  futex_wake(&hdr_->doorbell);
}

bool ShmControl::wait_done(int w, int64_t timeout_ms, int64_t* reply) {
  check(w);
  CtlCell& c = cells_[w];
  const int64_t deadline = timeout_ms < 0 ? -1 : now_ms() + timeout_ms;
  int spins = 0;
  for (;;) {
    uint32_t s = c.state.load(std::memory_order_acquire);
    if (s == kDone) {
      *reply = c.reply;
      c.state.store(kFree, std::memory_order_release);
      return true;
    }
    if (stopped()) throw std::runtime_error("ShmControl: parameter server stopped");
    if (spins < 64) {           // the owner usually answers within microseconds
      ++spins;
      std::this_thread::yield();
      continue;
    }
    int64_t left = -1;
    if (deadline >= 0) {
      left = deadline - now_ms();
      if (left <= 0) return false;
    }
    // short slices: a stop() raised while we sleep is seen within 50 ms even if its wake is lost
    futex_wait(&c.state, s, left < 0 ? 50 : std::min<int64_t>(left, 50));
  }
}

int ShmControl::wait_any(int64_t timeout_ms, int* workers, int64_t* steps, int cap) {
  const int64_t deadline = timeout_ms < 0 ? -1 : now_ms() + timeout_ms;
  const int n = (int)hdr_->n_workers;
  int spins = 0;
  for (;;) {
    if (stopped()) return -1;
    uint32_t bell = hdr_->doorbell.load(std::memory_order_acquire);
    int got = 0;
    for (int w = 0; w < n && got < cap; ++w) {
      uint32_t expect = kFull;
      if (cells_[w].state.compare_exchange_strong(expect, kTaken, std::memory_order_acq_rel)) {
        workers[got] = w;
        steps[got] = cells_[w].step;
        ++got;
      }
    }
    if (got) return got;
    if (spins < 64) {
      ++spins;
      std::this_thread::yield();
      continue;
    }
    int64_t left = -1;
    if (deadline >= 0) {
      left = deadline - now_ms();
      if (left <= 0) return 0;
    }
    futex_wait(&hdr_->doorbell, bell, left < 0 ? 50 : std::min<int64_t>(left, 50));
  }
}

void ShmControl::done(int w, int64_t reply) {
  check(w);
  CtlCell& c = cells_[w];
  c.reply = reply;
  c.state.store(kDone, std::memory_order_release);
  futex_wake(&c.state);
}

void ShmControl::stop() {
  hdr_->stop.store(1, std::memory_order_release);
  hdr_->doorbell.fetch_add(1, std::memory_order_acq_rel);
  futex_wake(&hdr_->doorbell);
  for (uint32_t w = 0; w < hdr_->n_workers; ++w) futex_wake(&cells_[w].state);
}

}  // namespace dtf
