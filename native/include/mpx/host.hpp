// Host-side runtime pieces shared by the HIP command-line programs:
// error checking with the reference's stderr contract, RAII device buffers,
// event timing with an explicit warm-up policy, fast stdin scanning and
// buffered %.10e output.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mpx/capi.h"
#include "../../src/cpu/cpu_kernels.h"

// Same stderr format as the reference's CSC macro (lab1/src/main.cu:5-13),
// naming HIP; the process exits with status 1.
#define HIP_CHECK(call)                                                                      \
    do {                                                                                     \
        hipError_t _st = (call);                                                             \
        if (_st != hipSuccess) {                                                             \
            std::fprintf(stderr, "[ERROR HIP] File: '%s'; Line: %i; Message: %s.\n", __FILE__, \
                         __LINE__, hipGetErrorString(_st));                                  \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

// libmpx entry points report through mpx_last_error().
#define MPX_CHECK(call)                                                                         \
    do {                                                                                        \
        int _rc = (call);                                                                       \
        if (_rc != 0) {                                                                         \
            std::fprintf(stderr, "[ERROR HIP] File: '%s'; Line: %i; Message: %s.\n", __FILE__, \
                         __LINE__, mpx_last_error());                                           \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

namespace mpx {
namespace host {

// ---- device memory ----
template <typename T>
class DeviceBuffer {
  public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(size_t n) : n_(n) {
        if (n) HIP_CHECK(hipMalloc(&p_, n * sizeof(T)));
    }
    ~DeviceBuffer() {
        if (p_) (void)hipFree(p_);
    }
    DeviceBuffer(const DeviceBuffer &) = delete;
    DeviceBuffer &operator=(const DeviceBuffer &) = delete;
    T *get() const { return p_; }
    size_t size() const { return n_; }

  private:
    T *p_ = nullptr;
    size_t n_ = 0;
};

// ---- timing ----
// Kernel-only timing like the reference (events bracket the launch only,
// reference lab2/src/to_plot.cu:101-120). MPX_TIMING selects the policy:
//   cold      : time the very first launch of the kernel (the reference's
//               methodology: one launch per process). Code objects are loaded
//               and the stream has dispatched once (init_stream_queue), as in
//               a CUDA context; the kernel's own first dispatch is timed;
//   warm      : one untimed warm-up launch, then time one launch (default);
//   median:N  : warm-up, then the median of N timed launches;
//   cold-lazy : cold without the code-object preload: the timed span also
//               holds HIP's lazy load of the kernel's module (CUDA 12's lazy
//               module loading, the closest match to how the reference's
//               published cold numbers were taken); the stream's first
//               dispatch still happens before the timer (CUDA creates its
//               queues with the context).
// MPX_WARMUP=W overrides the number of untimed launches (harness --warmup W).
struct TimingPolicy {
    bool warmup = true;
    int warmups = 1;
    int reps = 1;
    bool preload = true;  // mpx_preload_modules before timing
    static TimingPolicy from_env() {
        TimingPolicy p;
        const char *s = std::getenv("MPX_TIMING");
        if (!s || !*s || std::strcmp(s, "warm") == 0) {
        } else if (std::strcmp(s, "cold") == 0 || std::strcmp(s, "cold-lazy") == 0) {
            p.warmup = false;
            p.warmups = 0;
            p.preload = std::strcmp(s, "cold") == 0;
        } else if (std::strncmp(s, "median:", 7) == 0) {
            p.reps = std::max(1, std::atoi(s + 7));
        } else {
            std::fprintf(stderr, "[WARN] unknown MPX_TIMING='%s', using warm\n", s);
        }
        if (const char *w = std::getenv("MPX_WARMUP")) {
            p.warmups = std::max(0, std::atoi(w));
            p.warmup = p.warmups > 0;
        }
        return p;
    }
};

// Runtime set-up that CUDA performs at context creation but HIP defers to the
// first launch: loading each code object (~0.25 ms per module, measured with
// AMD_LOG_LEVEL=4, profiles/harness_vs_published.md) and the first dispatch on
// the stream. Both happen before the timer starts under every policy, 'cold'
// included ('cold-lazy' skips the preload): the measured kernel itself still
// runs for the first time.
// (HIP_ENABLE_DEFERRED_LOADING=0 would do the same, but HIP reads it before
// main(), so it only works when set by the caller's environment.)
__global__ void mpx_runtime_noop_kernel() {}
inline void init_stream_queue(hipStream_t stream, bool preload = true) {
    if (preload) MPX_CHECK(mpx_preload_modules());
    hipLaunchKernelGGL(mpx_runtime_noop_kernel, dim3(1), dim3(64), 0, stream);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(stream));
}

struct NoRestore {
    void operator()() const {}
};

// Runs `launch()` under the policy; returns kernel milliseconds. `restore()`
// runs before every launch, outside the event pair (in-place kernels whose
// warm-up would otherwise hand the timed launch already-processed data).
template <typename F, typename R = NoRestore>
float time_kernel(F &&launch, hipStream_t stream = nullptr, R &&restore = R{}) {
    const TimingPolicy pol = TimingPolicy::from_env();
    init_stream_queue(stream, pol.preload);
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    for (int i = 0; i < pol.warmups; ++i) {
        restore();
        launch();
        HIP_CHECK(hipStreamSynchronize(stream));
    }
    std::vector<float> ts;
    for (int i = 0; i < pol.reps; ++i) {
        restore();
        HIP_CHECK(hipEventRecord(a, stream));
        launch();
        HIP_CHECK(hipEventRecord(b, stream));
        HIP_CHECK(hipEventSynchronize(b));
        HIP_CHECK(hipGetLastError());
        float t = 0.0f;
        HIP_CHECK(hipEventElapsedTime(&t, a, b));
        ts.push_back(t);
    }
    HIP_CHECK(hipEventDestroy(a));
    HIP_CHECK(hipEventDestroy(b));
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

// ---- program start-up ----

// Harness geometries arrive on stdin only when both values are truthy
// (reference tester.py:113-121), so "tuned launch" is spelled as non-positive
// values: clamp them to 0, the C API's "choose for me".
inline void tuned_if_nonpositive(int &a, int &b) {
    if (a <= 0 || b <= 0) a = b = 0;
}

// ---- multi-device parts (MPX_NGPUS=N, harness --n_gpus N) ----
// The lab programs split their work into N parts; part p runs on device p
// with its own stream and events. The reported time is the max over parts of
// each part's kernel time — the parallel time of N GPUs. Fewer visible
// devices than parts is refused (exit 2) unless MPX_ALLOW_SHARED=1 rehearses
// the split on shared devices (part p on device p % visible).
inline int parts_from_env() {
    const char *s = std::getenv("MPX_NGPUS");
    const int n = s ? std::atoi(s) : 1;
    return n < 1 ? 1 : n;
}

class Parts {
  public:
    struct Part {
        int dev = 0;
        hipStream_t stream = nullptr;
        hipEvent_t a = nullptr, b = nullptr;
    };
    explicit Parts(int n) : p_(n) {
        int ndev = 0;
        HIP_CHECK(hipGetDeviceCount(&ndev));
        // an N-part time is an N-GPU time only on N devices: refuse to share
        // one unless asked to rehearse (MPX_ALLOW_SHARED=1)
        const char *shared = std::getenv("MPX_ALLOW_SHARED");
        if (n > ndev && !(shared && shared[0] == '1')) {
            std::fprintf(stderr, "[ERROR] MPX_NGPUS=%d but %d device(s) are visible (MPX_ALLOW_SHARED=1 to share)\n",
                         n, ndev);
            std::exit(2);
        }
        for (int i = 0; i < n; ++i) {
            p_[i].dev = i % ndev;
            HIP_CHECK(hipSetDevice(p_[i].dev));
            HIP_CHECK(hipStreamCreateWithFlags(&p_[i].stream, hipStreamNonBlocking));
            HIP_CHECK(hipEventCreate(&p_[i].a));
            HIP_CHECK(hipEventCreate(&p_[i].b));
        }
    }
    ~Parts() {
        for (auto &q : p_) {
            (void)hipSetDevice(q.dev);
            (void)hipEventDestroy(q.a);
            (void)hipEventDestroy(q.b);
            (void)hipStreamDestroy(q.stream);
        }
    }
    Parts(const Parts &) = delete;
    Parts &operator=(const Parts &) = delete;
    int size() const { return (int)p_.size(); }
    const Part &operator[](int i) const { return p_[i]; }
    void use(int i) const { HIP_CHECK(hipSetDevice(p_[i].dev)); }
    void sync_all() const {
        for (int i = 0; i < size(); ++i) {
            use(i);
            HIP_CHECK(hipStreamSynchronize(p_[i].stream));
        }
    }
    // launch(i, stream) queues part i; returns kernel ms under MPX_TIMING
    template <typename F>
    float time(F &&launch) const {
        const TimingPolicy pol = TimingPolicy::from_env();
        for (int i = 0; i < size(); ++i) {
            use(i);
            // the parts' streams are non-blocking: a pageable hipMemcpy that
            // filled the inputs may return before its last DMA chunk lands, and
            // nothing orders it before this stream's kernels — drain the device
            HIP_CHECK(hipDeviceSynchronize());
            init_stream_queue(p_[i].stream, pol.preload);
        }
        for (int w = 0; w < pol.warmups; ++w) {
            for (int i = 0; i < size(); ++i) {
                use(i);
                launch(i, p_[i].stream);
            }
            sync_all();
        }
        std::vector<float> ts;
        for (int r = 0; r < pol.reps; ++r) {
            for (int i = 0; i < size(); ++i) {
                use(i);
                HIP_CHECK(hipEventRecord(p_[i].a, p_[i].stream));
                launch(i, p_[i].stream);
                HIP_CHECK(hipEventRecord(p_[i].b, p_[i].stream));
            }
            float worst = 0.0f;
            for (int i = 0; i < size(); ++i) {
                use(i);
                HIP_CHECK(hipEventSynchronize(p_[i].b));
                HIP_CHECK(hipGetLastError());
                float t = 0.0f;
                HIP_CHECK(hipEventElapsedTime(&t, p_[i].a, p_[i].b));
                worst = std::max(worst, t);
            }
            ts.push_back(worst);
        }
        std::sort(ts.begin(), ts.end());
        return ts[ts.size() / 2];
    }

  private:
    std::vector<Part> p_;
};

// [begin, end) of part i of n over `total` items, boundaries multiples of `align`
inline void part_range(int64_t total, int n, int i, int64_t align, int64_t &begin, int64_t &end) {
    const int64_t per = ((total + n - 1) / n + align - 1) / align * align;
    begin = std::min<int64_t>(total, per * i);
    end = std::min<int64_t>(total, begin + per);
}

// ---- stdin ----
// Whole-stream tokenizer: the reference parses up to 2*2^25 doubles with one
// scanf each (lab1/src/main.cu:46-52); reading stdin once and strtod-ing the
// buffer is an order of magnitude faster and accepts the same text.
class Scanner {
  public:
    Scanner() {
        std::vector<char> chunk(1 << 20);
        size_t got;
        while ((got = std::fread(chunk.data(), 1, chunk.size(), stdin)) > 0) buf_.append(chunk.data(), got);
        pos_ = 0;
    }
    bool next_token(std::string &tok) {
        skip_ws();
        if (pos_ >= buf_.size()) return false;
        const size_t st = pos_;
        while (pos_ < buf_.size() && !is_ws(buf_[pos_])) ++pos_;
        tok.assign(buf_, st, pos_ - st);
        return true;
    }
    bool next_int(int &v) {
        skip_ws();
        if (pos_ >= buf_.size()) return false;
        char *end = nullptr;
        const long x = std::strtol(buf_.c_str() + pos_, &end, 10);
        if (end == buf_.c_str() + pos_) return false;
        pos_ = end - buf_.c_str();
        v = (int)x;
        return true;
    }
    // the next `count` numbers in parallel (libmpx's OpenMP mpx_parse_doubles:
    // one strtod per token, so the values are those of next_double)
    int64_t next_doubles(double *out, int64_t count) {
        size_t end = pos_;
        const int64_t got = mpx_parse_doubles(buf_.c_str(), buf_.size(), pos_, count, out, &end);
        if (got == count) pos_ = end;
        return got;
    }
    bool next_double(double &v) {
        skip_ws();
        if (pos_ >= buf_.size()) return false;
        char *end = nullptr;
        v = std::strtod(buf_.c_str() + pos_, &end);
        if (end == buf_.c_str() + pos_) return false;
        pos_ = end - buf_.c_str();
        return true;
    }

  private:
    static bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\f' || c == '\v'; }
    void skip_ws() {
        while (pos_ < buf_.size() && is_ws(buf_[pos_])) ++pos_;
    }
    std::string buf_;
    size_t pos_ = 0;
};

// ---- stdout ----
// "%.10e " writer (reference lab1/src/to_plot.cu:86-88 prints one printf per
// element): formatted in parallel per thread range (mpx_format_e10), written
// in order with one fwrite.
inline void print_e10(const double *v, int64_t n) {
    size_t len = 0;
    char *buf = mpx_format_e10(v, n, &len);
    if (!buf && n) {
        std::fprintf(stderr, "[ERROR CPU] out of memory formatting %lld values\n", (long long)n);
        std::exit(1);
    }
    if (len) std::fwrite(buf, 1, len, stdout);
    std::free(buf);
}

}  // namespace host
}  // namespace mpx
