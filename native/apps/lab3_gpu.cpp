// lab3 GPU program: per-pixel Mahalanobis maximum-likelihood classification,
// stdin/stdout contract of the reference.
//
//   benchmark personality ("to_plot_hip_exe"):
//     stdin  "<blocks>\n<threads>\n<in.data>\n<out.data>\n<nc>\n<np x y x y ...>\n..."
//     stdout "HIP execution time: <X ms>\n" (reference lab3/src/to_plot.cu:76-117,174)
//   submission personality (-DMPX_SUBMISSION, "hip_exe"): no geometry, no output line.
// Output: the input image with alpha = class index (255 when every distance is NaN).
// MPX_LAB3_PATH = direct (default, geometry honoured) | fast | mfma | mfma64 | auto.
// MPX_NGPUS=N shards the pixels over N devices (harness --n_gpus N).
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "mpx/cio.h"
#include "mpx/common.h"
#include "mpx/host.hpp"

int main() {
    using namespace mpx::host;
    Scanner in;
    int blocks = 256, threads = 256;  // reference submission launch (lab3/src/main.cu:32-33)
#ifndef MPX_SUBMISSION
    if (!in.next_int(blocks) || !in.next_int(threads)) {
        std::fprintf(stderr, "[ERROR CPU] expected <blocks> <threads> on stdin\n");
        return 1;
    }
    tuned_if_nonpositive(blocks, threads);
#endif
    int path = MPX_CLS_DIRECT;
    if (const char *e = std::getenv("MPX_LAB3_PATH")) {
        if (!std::strcmp(e, "mfma")) path = MPX_CLS_MFMA;
        else if (!std::strcmp(e, "auto")) path = MPX_CLS_AUTO;
        else if (!std::strcmp(e, "fast")) path = MPX_CLS_FAST;
        else if (!std::strcmp(e, "mfma64")) path = MPX_CLS_MFMA64;
        else if (!std::strcmp(e, "mfma8")) path = MPX_CLS_MFMA8;
        else if (!std::strcmp(e, "mfma16")) path = MPX_CLS_MFMA16;
    }
    std::string in_path, out_path;
    if (!in.next_token(in_path) || !in.next_token(out_path)) {
        std::fprintf(stderr, "[ERROR CPU] expected input and output paths on stdin\n");
        return 1;
    }
    int w = 0, h = 0;
    uint32_t *img = mpx_read_data_image(in_path.c_str(), &w, &h);
    if (!img) return 1;
    const int64_t npix = (int64_t)w * h;

    int nc = 0;
    if (!in.next_int(nc) || nc < 1 || nc > MPX_MAX_CLASSES) {
        std::fprintf(stderr, "[ERROR CPU] expected 1 <= nc <= %d\n", MPX_MAX_CLASSES);
        return 1;
    }
    std::vector<int> np(nc), coords;
    for (int c = 0; c < nc; ++c) {
        if (!in.next_int(np[c]) || np[c] < 1) {
            std::fprintf(stderr, "[ERROR CPU] class %d: expected a positive point count\n", c);
            return 1;
        }
        for (int i = 0; i < 2 * np[c]; ++i) {
            int v;
            if (!in.next_int(v)) {
                std::fprintf(stderr, "[ERROR CPU] class %d: truncated coordinate list\n", c);
                return 1;
            }
            coords.push_back(v);
        }
    }
    std::vector<double> mu(3 * nc), inv(9 * nc);
    MPX_CHECK(mpx_class_stats(img, w, h, nc, np.data(), coords.data(), mu.data(), inv.data()));

    const int nparts = parts_from_env();
    float ms = 0.0f;
    if (nparts == 1) {
        DeviceBuffer<uint32_t> dimg(npix);
        HIP_CHECK(hipMemcpy(dimg.get(), img, npix * 4, hipMemcpyHostToDevice));
        ms = time_kernel([&] {
            MPX_CHECK(mpx_classify(dimg.get(), npix, nc, mu.data(), inv.data(), blocks, threads, path, nullptr));
        });
        HIP_CHECK(hipMemcpy(img, dimg.get(), npix * 4, hipMemcpyDeviceToHost));
    } else {
        // MPX_NGPUS = N: pixel shards (128-pixel aligned), class statistics
        // computed once on the host and passed to every device's launch
        Parts parts(nparts);
        std::vector<std::unique_ptr<DeviceBuffer<uint32_t>>> d(nparts);
        std::vector<int64_t> lo(nparts), hi(nparts);
        for (int i = 0; i < nparts; ++i) {
            part_range(npix, nparts, i, 128, lo[i], hi[i]);
            parts.use(i);
            d[i].reset(new DeviceBuffer<uint32_t>(hi[i] - lo[i]));
            if (hi[i] > lo[i])
                HIP_CHECK(hipMemcpy(d[i]->get(), img + lo[i], (hi[i] - lo[i]) * 4, hipMemcpyHostToDevice));
        }
        ms = parts.time([&](int i, hipStream_t st) {
            MPX_CHECK(mpx_classify(d[i]->get(), hi[i] - lo[i], nc, mu.data(), inv.data(), blocks, threads, path, st));
        });
        for (int i = 0; i < nparts; ++i) {
            parts.use(i);
            if (hi[i] > lo[i])
                HIP_CHECK(hipMemcpy(img + lo[i], d[i]->get(), (hi[i] - lo[i]) * 4, hipMemcpyDeviceToHost));
        }
    }
    const int rc = mpx_write_data_image(out_path.c_str(), img, w, h);
    std::free(img);
    if (rc) return 1;
#ifndef MPX_SUBMISSION
    std::printf("HIP execution time: <%f ms>\n", ms);
#else
    (void)ms;
#endif
    return 0;
}
