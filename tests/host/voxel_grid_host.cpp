// Host harness for csrc/voxel_grid.hpp (tests/test_voxel_grid_host.py): the device kernels' binning,
// compiled for the host.  stdin: int64 n, double voxel, float32 xyz[n][3]; stdout: int64 ok, nx, ny,
// nz, then int64 bins[n][3] (-1 outside) and uint32 keys[n].
#include <stdio.h>
#include <vector>

#include "voxel_grid.hpp"

int main()
{
    int64_t n;
    double v;
    if (fread(&n, 8, 1, stdin) != 1 || fread(&v, 8, 1, stdin) != 1) return 2;
    std::vector<float> p((size_t)n * 3);
    if (fread(p.data(), 4, p.size(), stdin) != p.size()) return 2;
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = hi[a] = p[a];
        for (int64_t i = 0; i < n; ++i) {
            lo[a] = p[3 * i + a] < lo[a] ? p[3 * i + a] : lo[a];
            hi[a] = p[3 * i + a] > hi[a] ? p[3 * i + a] : hi[a];
        }
    }
    const lidar_vox::Grid g = lidar_vox::make_grid(lo, hi, v);
    const int64_t head[4] = {g.ok ? 1 : 0, g.ax[0].nb, g.ax[1].nb, g.ax[2].nb};
    fwrite(head, 8, 4, stdout);
    if (!g.ok) return 0;
    std::vector<int64_t> b((size_t)n * 3);
    std::vector<uint32_t> k((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        for (int a = 0; a < 3; ++a) b[3 * i + a] = lidar_vox::bin(g.ax[a], (double)p[3 * i + a]);
        k[i] = lidar_vox::key(g, p[3 * i], p[3 * i + 1], p[3 * i + 2]);
    }
    fwrite(b.data(), 8, b.size(), stdout);
    fwrite(k.data(), 4, k.size(), stdout);
    return 0;
}
