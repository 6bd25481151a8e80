// lab1 GPU program: c = a - b over fp64 vectors, stdin/stdout contract of
// the reference.
//
//   benchmark personality (default build, "to_plot_hip_exe"):
//     stdin  "<grid>\n<block>\n<n>\n<a0 .. a(n-1)>\n<b0 .. b(n-1)>"
//     stdout "HIP execution time: <X ms>\n" then n x "%.10e "
//     (reference lab1/src/to_plot.cu:36-40,72,82,86-88)
//   submission personality (-DMPX_SUBMISSION, "hip_exe"):
//     no geometry lines, fixed launch, values only (reference lab1/src/main.cu).
// Geometry 0 0 selects the MI355X-tuned launch. MPX_NGPUS=N shards the vectors
// over N devices (harness --n_gpus N); the reported time is the slowest shard.
#include <memory>
#include <vector>

#include "mpx/host.hpp"

int main() {
    using namespace mpx::host;
    Scanner in;
    int grid = 512, block = 512;  // reference submission launch <<<512, 512>>>
#ifndef MPX_SUBMISSION
    if (!in.next_int(grid) || !in.next_int(block)) {
        std::fprintf(stderr, "[ERROR CPU] expected launch geometry <grid> <block> on stdin\n");
        return 1;
    }
    tuned_if_nonpositive(grid, block);
#endif
    int n = 0;
    if (!in.next_int(n) || n < 0) {
        std::fprintf(stderr, "[ERROR CPU] expected vector size on stdin\n");
        return 1;
    }
    std::vector<double> a(n), b(n), c(n);
    // both vectors parsed in parallel (host.hpp Scanner::next_doubles)
    if (const int64_t got = in.next_doubles(a.data(), n); got != n) {
        std::fprintf(stderr, "[ERROR CPU] first vector: expected %d values, got %lld\n", n, (long long)got);
        return 1;
    }
    if (const int64_t got = in.next_doubles(b.data(), n); got != n) {
        std::fprintf(stderr, "[ERROR CPU] second vector: expected %d values, got %lld\n", n, (long long)got);
        return 1;
    }

    const int nparts = parts_from_env();
    float ms = 0.0f;
    if (nparts == 1) {
        DeviceBuffer<double> da(n), db(n), dc(n);
        if (n) {
            HIP_CHECK(hipMemcpy(da.get(), a.data(), sizeof(double) * n, hipMemcpyHostToDevice));
            HIP_CHECK(hipMemcpy(db.get(), b.data(), sizeof(double) * n, hipMemcpyHostToDevice));
        }
        ms = time_kernel([&] { MPX_CHECK(mpx_vsub_f64(da.get(), db.get(), dc.get(), n, grid, block, nullptr)); });
        if (n) HIP_CHECK(hipMemcpy(c.data(), dc.get(), sizeof(double) * n, hipMemcpyDeviceToHost));
    } else {
        // MPX_NGPUS = N: contiguous shards, one per device, the geometry per shard
        Parts parts(nparts);
        std::vector<std::unique_ptr<DeviceBuffer<double>>> A(nparts), B(nparts), C(nparts);
        std::vector<int64_t> lo(nparts), hi(nparts);
        for (int i = 0; i < nparts; ++i) {
            part_range(n, nparts, i, 2, lo[i], hi[i]);
            const int64_t m = hi[i] - lo[i];
            parts.use(i);
            A[i].reset(new DeviceBuffer<double>(m));
            B[i].reset(new DeviceBuffer<double>(m));
            C[i].reset(new DeviceBuffer<double>(m));
            if (m) {
                HIP_CHECK(hipMemcpy(A[i]->get(), a.data() + lo[i], sizeof(double) * m, hipMemcpyHostToDevice));
                HIP_CHECK(hipMemcpy(B[i]->get(), b.data() + lo[i], sizeof(double) * m, hipMemcpyHostToDevice));
            }
        }
        ms = parts.time([&](int i, hipStream_t st) {
            MPX_CHECK(mpx_vsub_f64(A[i]->get(), B[i]->get(), C[i]->get(), hi[i] - lo[i], grid, block, st));
        });
        for (int i = 0; i < nparts; ++i) {
            parts.use(i);
            if (hi[i] > lo[i])
                HIP_CHECK(hipMemcpy(c.data() + lo[i], C[i]->get(), sizeof(double) * (hi[i] - lo[i]),
                                    hipMemcpyDeviceToHost));
        }
    }
#ifndef MPX_SUBMISSION
    std::printf("HIP execution time: <%f ms>\n", ms);
#else
    (void)ms;
#endif
    std::fflush(stdout);
    print_e10(c.data(), n);
    return 0;
}
