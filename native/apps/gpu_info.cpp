// gpu_info: device properties of every visible GPU (reference
// gpu_info/src/main.cu prints device 0 unchecked; this checks every call and
// adds the CDNA facts — gfx arch, wave size, LDS per CU, L2).
#include <cstdio>

#include "mpx/host.hpp"

int main() {
    int n = 0;
    MPX_CHECK(mpx_device_count(&n));
    if (n == 0) {
        std::fprintf(stderr, "[ERROR HIP] no HIP devices visible\n");
        return 1;
    }
    for (int d = 0; d < n; ++d) {
        char buf[4096];
        MPX_CHECK(mpx_device_report(d, buf, sizeof(buf)));
        if (n > 1) std::printf("Device %d\n", d);
        std::fputs(buf, stdout);
    }
    return 0;
}
