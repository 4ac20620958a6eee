// mof_hostio.h -- host <-> HBM staging for the host-pointer form of
// mof_solve_range (the drop-in's path: S3 hands numpy arrays in and gets
// numpy arrays back, compute_optical_flow.py:152-194).
//
// Pageable caller memory is moved through a small ring of pinned chunks on
// a copy stream of its own: a pool of host threads copies chunk c+1 into
// pinned memory while the DMA engine moves chunk c, so a batch's input
// upload and the previous batch's V download run beside the solve of the
// current batch instead of before and after it.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mof {

// Fixed set of worker threads running one parallel loop at a time.
class CopyPool {
  public:
    explicit CopyPool(int32_t threads);
    ~CopyPool();
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;
    int32_t size() const { return (int32_t)workers_.size() + 1; }
    // body(t, a, b) for the T contiguous slices [a, b) of [0, n); the calling
    // thread runs slice 0.
    void run(int64_t n, const std::function<void(int32_t, int64_t, int64_t)> &body);
    // memcpy in parallel slices
    void copy(void *dst, const void *src, size_t bytes);

  private:
    void loop(int32_t t);
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int32_t, int64_t, int64_t)> *job_ = nullptr;
    int64_t n_ = 0;
    uint64_t gen_ = 0;
    int32_t pending_ = 0;
    bool stop_ = false;
};

// Pinned chunk ring + copy stream of one mesh handle (created on its device).
class HostStage {
  public:
    HostStage(size_t chunk_bytes, int32_t threads);
    ~HostStage();
    HostStage(const HostStage &) = delete;
    HostStage &operator=(const HostStage &) = delete;
    hipStream_t stream() const { return cs_; }
    size_t chunk() const { return chunk_; }
    // Enqueue pageable src -> device dst on the copy stream (returns once
    // every chunk is in pinned memory and its DMA is queued).
    void h2d(void *dst_dev, const void *src, size_t bytes);
    // Device src -> pageable dst through the ring; returns when dst holds
    // the data. The copy stream first waits for `ready` (may be null).
    void d2h(void *dst, const void *src_dev, size_t bytes, hipEvent_t ready);

  private:
    int32_t take_slot();  // next ring slot, its previous DMA finished
    static constexpr int kSlots = 4;
    size_t chunk_;
    hipStream_t cs_ = nullptr;
    void *pin_[kSlots] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_[kSlots] = {nullptr, nullptr, nullptr, nullptr};
    bool used_[kSlots] = {false, false, false, false};
    int32_t next_ = 0;
    CopyPool pool_;
};

// host threads for staging copies: $MOF_IO_THREADS, else $OMP_NUM_THREADS,
// else the host's cores; at most 16 per handle
int32_t stage_threads();

}  // namespace mof
