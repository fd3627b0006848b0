// Host harness for csrc/voxel_grid.hpp (tests/test_voxel_grid_host.py): the device kernels' binning,
// compiled for the host.  stdin: int64 n, double voxel, float32 xyz[n][3]; stdout: int64 ok, nx, ny,
// nz, then int64 bins[n][3] (-1 outside) and uint32 keys[n], then the keys launch's float binning
// (voxel_batch.hip: thresholds ru_float(edge) per axis, the spacing guess, the search on a miss): int64
// tab (1 when every axis' table applies, else the launch runs key() and so does this) and int64
// fbins[n][3], computed the same way as the launch.
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

    lidar_vox::FAxis fa[3];
    std::vector<float> E[3];
    int64_t tab = 1;
    for (int a = 0; a < 3; ++a) {
        fa[a] = lidar_vox::faxis(g.ax[a], lidar_vox::kTabEdges);
        tab = tab && fa[a].ok;
    }
    if (tab)
        for (int a = 0; a < 3; ++a) {  // -inf, the thresholds, +inf (as the launch's LDS tables)
            E[a].push_back(-INFINITY);
            for (int i = 0; i < fa[a].L; ++i) E[a].push_back(lidar_vox::ru_float(lidar_vox::edge(g.ax[a], i)));
            E[a].push_back(INFINITY);
        }
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            const float q = p[3 * i + a];
            if (!tab) {
                b[3 * i + a] = lidar_vox::bin(g.ax[a], (double)q);
                continue;
            }
            int c = lidar_vox::bin_tab_c(E[a].data() + 1, fa[a].L, q, fa[a].s0, fa[a].inv);
            if (c < 0) c = lidar_vox::bin_tab_search(E[a].data() + 1, fa[a].L, q);
            const uint32_t bb = lidar_vox::bin_of_c(c, q, fa[a].lastf, fa[a].L);
            b[3 * i + a] = bb == lidar_vox::kOutside ? -1 : (int64_t)bb;
        }
    fwrite(&tab, 8, 1, stdout);
    fwrite(b.data(), 8, b.size(), stdout);
    return 0;
}
