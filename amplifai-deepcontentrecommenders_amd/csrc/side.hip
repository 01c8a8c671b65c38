// A second host thread that issues a step's side-stream work (the user tower, the weight-gradient
// launches, the late Adam, a plan's next-step inputs) while the calling thread issues the caller's
// stream chain. Each HIP launch costs the issuing thread ~2.6 µs and each record/wait pair ~2.8 µs
// on MI355X / ROCm 7.2; two threads issuing to different streams reach ~1.7 µs per launch of wall
// time (profiles/tools/mtlaunch.cpp, measured), so a step's host issue time becomes roughly the
// longer of the two parts instead of their sum.
//
// Ordering is the same as with one thread: the caller posts a side closure only after it has
// recorded (or bound to a launch) every event the closure waits on, and waits for a closure's
// completion (side_wait) before it waits on an event the closure records. Closures run in post
// order (FIFO), so side streams see their work in the single-thread issue order.
//
// One worker per device's SidePool, spinning while work is frequent (a futex wake-up costs tens of
// µs) and parked on a condition variable after ~50 ms idle. DCUE_SIDE_THREAD=0 issues everything
// on the calling thread (A/B). Stream capture (graph plans) always issues inline.
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include "dcue_internal.h"

namespace dcue {

namespace {
thread_local bool t_side_worker = false;

class SideIssuer {
 public:
  explicit SideIssuer(int dev) : dev_(dev) { th_ = std::thread([this] { loop(); }); }
  ~SideIssuer() {
    stop_.store(true, std::memory_order_release);
    wake();
    if (th_.joinable()) th_.join();
  }
  // Any host thread of the process may post (one issuer per device): posts are serialised. The
  // head store and the parked load are sequentially consistent, as are the worker's parked store
  // and its head load: either this post sees the worker parked and wakes it, or the worker's check
  // before sleeping sees the new head.
  uint64_t post(std::function<int()> fn) {
    std::lock_guard<std::mutex> lk(post_mu_);
    const uint64_t h = head_.load(std::memory_order_relaxed);
    while (h - done_.load(std::memory_order_acquire) >= kQ) __builtin_ia32_pause();
    q_[h % kQ] = std::move(fn);
    head_.store(h + 1, std::memory_order_seq_cst);
    if (parked_.load(std::memory_order_seq_cst)) wake();
    return h + 1;
  }
  int wait(uint64_t seq) {
    while (done_.load(std::memory_order_acquire) < seq) __builtin_ia32_pause();
    return err_.exchange(0, std::memory_order_acq_rel);
  }
  uint64_t posted() const { return head_.load(std::memory_order_relaxed); }

 private:
  static constexpr uint64_t kQ = 64;
  void wake() {
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_one();
  }
  void loop() {
    t_side_worker = true;
    if (hipSetDevice(dev_) != hipSuccess) err_.store(DCUE_ERR_HIP);
    auto idle_since = std::chrono::steady_clock::now();
    unsigned spins = 0;
    bool worked = false;  // a closure ran since the idle clock was last started
    while (!stop_.load(std::memory_order_acquire)) {
      const uint64_t d = done_.load(std::memory_order_relaxed);
      if (d < head_.load(std::memory_order_acquire)) {
        const int st = q_[d % kQ]();
        q_[d % kQ] = nullptr;
        if (st) {
          int zero = 0;
          err_.compare_exchange_strong(zero, st, std::memory_order_acq_rel);
        }
        done_.store(d + 1, std::memory_order_release);
        spins = 0;
        worked = true;
        continue;
      }
      __builtin_ia32_pause();
      if (++spins < 4096) continue;
      spins = 0;
      const auto now = std::chrono::steady_clock::now();
      if (worked) {  // idle time counts from the last closure, not from the last wake-up (round 6:
        worked = false;  // a stale clock parked the worker ~100 us into every idle stretch of a
        idle_since = now;  // running step loop, and each post then paid a futex wake-up)
      }
      if (now - idle_since < std::chrono::milliseconds(50)) {
        std::this_thread::yield();
        continue;
      }
      std::unique_lock<std::mutex> lk(mu_);
      parked_.store(true, std::memory_order_seq_cst);
      cv_.wait_for(lk, std::chrono::milliseconds(100), [this] {
        return stop_.load(std::memory_order_acquire) ||
               done_.load(std::memory_order_relaxed) < head_.load(std::memory_order_seq_cst);
      });
      parked_.store(false, std::memory_order_seq_cst);
      idle_since = std::chrono::steady_clock::now();
    }
  }
  int dev_;
  std::thread th_;
  std::function<int()> q_[kQ];
  std::atomic<uint64_t> head_{0}, done_{0};
  std::atomic<int> err_{0};
  std::atomic<bool> stop_{false}, parked_{false};
  std::mutex mu_, post_mu_;
  std::condition_variable cv_;
};

bool side_thread_on() {
  static const bool on = [] {
    const char* e = getenv("DCUE_SIDE_THREAD");
    return !(e && e[0] == '0');
  }();
  return on;
}

SideIssuer* issuer_for_device() {
  static std::atomic<SideIssuer*> per_dev[64] = {};
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  SideIssuer* p = per_dev[dev].load(std::memory_order_acquire);
  if (!p) {
    std::lock_guard<std::mutex> lk(mu);
    // never destroyed: the worker parks when idle and ends with the process
    p = per_dev[dev].load(std::memory_order_relaxed);
    if (!p) {
      p = new SideIssuer(dev);
      per_dev[dev].store(p, std::memory_order_release);
    }
  }
  return p;
}
}  // namespace

bool on_side_worker() { return t_side_worker; }

SideQueue::SideQueue(bool enable) {
  if (enable && side_thread_on() && !capturing_step() && !t_side_worker) impl_ = issuer_for_device();
}

SideQueue::~SideQueue() {
  if (impl_ && last_) static_cast<SideIssuer*>(impl_)->wait(last_);
}

uint64_t SideQueue::run(std::function<int()> fn, int* inline_status) {
  if (!impl_) {
    *inline_status = fn();
    return 0;
  }
  last_ = static_cast<SideIssuer*>(impl_)->post(std::move(fn));
  return last_;
}

int SideQueue::wait(uint64_t seq) {
  if (!impl_ || !seq) return DCUE_OK;
  return static_cast<SideIssuer*>(impl_)->wait(seq);
}

int SideQueue::drain() { return wait(last_); }

}  // namespace dcue
