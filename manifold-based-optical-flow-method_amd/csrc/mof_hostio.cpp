// mof_hostio.cpp -- pinned-ring staging between pageable host memory and HBM
// (mof_hostio.h). Host code only; the DMA runs on a copy stream per handle.
#include "mof_hostio.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "mof_internal.h"

namespace mof {

CopyPool::CopyPool(int32_t threads) {
    for (int32_t t = 1; t < std::max(1, threads); ++t) workers_.emplace_back([this, t] { loop(t); });
}

CopyPool::~CopyPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto &w : workers_) w.join();
}

void CopyPool::loop(int32_t t) {
    uint64_t seen = 0;
    for (;;) {
        const std::function<void(int32_t, int64_t, int64_t)> *job;
        int64_t n;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            job = job_;
            n = n_;
        }
        const int64_t T = size();
        (*job)(t, n * t / T, n * (t + 1) / T);
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_cv_.notify_one();
        }
    }
}

void CopyPool::run(int64_t n, const std::function<void(int32_t, int64_t, int64_t)> &body) {
    const int64_t T = size();
    if (T == 1 || n < T) {
        body(0, 0, n);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = &body;
        n_ = n;
        pending_ = (int32_t)workers_.size();
        ++gen_;
    }
    cv_.notify_all();
    body(0, 0, n / T);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
}

void CopyPool::copy(void *dst, const void *src, size_t bytes) {
    // 64-B aligned slices (whole cache lines per thread)
    const int64_t lines = (int64_t)((bytes + 63) / 64);
    if (bytes < ((size_t)1 << 20)) {
        std::memcpy(dst, src, bytes);
        return;
    }
    run(lines, [&](int32_t, int64_t a, int64_t b) {
        const size_t o = (size_t)a * 64, e = std::min(bytes, (size_t)b * 64);
        if (e > o) std::memcpy((char *)dst + o, (const char *)src + o, e - o);
    });
}

int32_t stage_threads() {
    if (const int32_t t = knob_threads(16)) return t;
    const unsigned hc = std::thread::hardware_concurrency();
    return (int32_t)std::min(16u, std::max(1u, hc));
}

HostStage::HostStage(size_t chunk_bytes, int32_t threads) : chunk_(chunk_bytes), pool_(threads) {
    MOF_HIP(hipStreamCreateWithFlags(&cs_, hipStreamNonBlocking));
    for (int k = 0; k < kSlots; ++k) {
        MOF_HIP(hipHostMalloc(&pin_[k], chunk_, hipHostMallocDefault));
        MOF_HIP(hipEventCreateWithFlags(&ev_[k], hipEventDisableTiming));
    }
}

HostStage::~HostStage() {
    if (cs_) (void)hipStreamSynchronize(cs_);
    for (int k = 0; k < kSlots; ++k) {
        if (ev_[k]) (void)hipEventDestroy(ev_[k]);
        if (pin_[k]) (void)hipHostFree(pin_[k]);
    }
    if (cs_) (void)hipStreamDestroy(cs_);
}

int32_t HostStage::take_slot() {
    const int32_t k = next_;
    next_ = (next_ + 1) % kSlots;
    if (used_[k]) MOF_HIP(hipEventSynchronize(ev_[k]));
    used_[k] = false;
    return k;
}

void HostStage::h2d(void *dst_dev, const void *src, size_t bytes) {
    for (size_t o = 0; o < bytes; o += chunk_) {
        const size_t len = std::min(chunk_, bytes - o);
        const int32_t k = take_slot();
        pool_.copy(pin_[k], (const char *)src + o, len);
        MOF_HIP(hipMemcpyAsync((char *)dst_dev + o, pin_[k], len, hipMemcpyHostToDevice, cs_));
        MOF_HIP(hipEventRecord(ev_[k], cs_));
        used_[k] = true;
    }
}

void HostStage::d2h(void *dst, const void *src_dev, size_t bytes, hipEvent_t ready) {
    if (ready) MOF_HIP(hipStreamWaitEvent(cs_, ready, 0));
    const size_t nch = (bytes + chunk_ - 1) / chunk_;
    // keep up to kSlots - 1 chunk DMAs in flight ahead of the host copy
    std::vector<int32_t> slot(nch);
    size_t issued = 0;
    auto issue = [&](size_t c) {
        const size_t o = c * chunk_, len = std::min(chunk_, bytes - o);
        const int32_t k = take_slot();
        MOF_HIP(hipMemcpyAsync(pin_[k], (const char *)src_dev + o, len, hipMemcpyDeviceToHost, cs_));
        MOF_HIP(hipEventRecord(ev_[k], cs_));
        used_[k] = true;
        slot[c] = k;
    };
    for (size_t c = 0; c < nch; ++c) {
        while (issued < nch && issued < c + kSlots - 1) issue(issued++);
        const int32_t k = slot[c];
        const size_t o = c * chunk_, len = std::min(chunk_, bytes - o);
        MOF_HIP(hipEventSynchronize(ev_[k]));
        used_[k] = false;
        pool_.copy((char *)dst + o, pin_[k], len);
    }
}

}  // namespace mof
