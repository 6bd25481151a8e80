"""Debug probe: band kernel (forced) vs the CPU reference on small images;
prints, per filter and shape, how many pixels differ and where (column mod 4,
lane, first rows)."""
import torch

from cuda_mpi_openmp_amd import _native, ops
from tests.helpers import rand_img

L = _native.lib()
old = L.mpx_conv_set_band_min(0)
for filt in ("roberts", "sobel3", "sobel5", "gauss5", "log5", "sobel5_dense"):
    f = ops.get_filter(filt)
    for w in (4, 8, 252, 256, 260, 512):
        for h in (1, 2, 5, 17):
            img = rand_img(h, w, seed=w + h)
            g = ops.conv(img.to("cuda"), f).cpu()
            c = ops.conv(img, f)
            bad = (g[..., 0] != c[..., 0]).nonzero()
            if len(bad):
                cols = bad[:, -1]
                print(f"{filt} h={h} w={w}: {len(bad)} bad; col%4 {torch.bincount(cols % 4, minlength=4).tolist()} "
                      f"cols {sorted(set(cols.tolist()))[:12]} rows {sorted(set(bad[:, -2].tolist()))[:6]}", flush=True)
L.mpx_conv_set_band_min(old)
print("done")
