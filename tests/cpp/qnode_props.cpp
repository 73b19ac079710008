// Property check of tri_qnode.h (the 16-B quantized triangle-accelerator nodes): for random
// roots and child boxes -- magnitudes from 1e-30 to 1e6, denormals, signed zeros, boxes on
// and off the grid, degenerate (flat) boxes -- the decoded box (the kernel's exact fma)
// contains the stored box on every axis, the grid decode is exact (origin + q * scale equals
// the double-precision value), and the link word round-trips.
// usage: qnode_props <cases>  -> "ok <cases> <boxes>" or the first failure
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "tri_qnode.h"

int main(int argc, char** argv) {
    const long cases = argc > 1 ? atol(argv[1]) : 2000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> u01(0.0, 1.0);
    long boxes = 0;
    for (long c = 0; c < cases; c++) {
        // a root box at some scale and offset
        const double scale = std::pow(10.0, -30.0 + 36.0 * u01(rng));
        const double off = (u01(rng) < 0.5 ? 0.0 : (u01(rng) - 0.5) * 1e3 * scale * (u01(rng) < 0.1 ? 1e3 : 1.0));
        SphereBvhNode root{};
        for (int k = 0; k < 3; k++) {
            double lo = off + (u01(rng) - 0.5) * scale, hi = lo + u01(rng) * scale;
            if (u01(rng) < 0.05) hi = lo;  // flat
            root.bmin[k] = std::nextafter((float)lo, -INFINITY);
            root.bmax[k] = std::nextafter((float)hi, INFINITY);
        }
        root.leaf = kSphereBvhInternal;
        root.skip = 7;
        const TriQGrid g = tri_qgrid(root);
        if (!g.valid) continue;
        for (int b = 0; b < 64; b++) {
            SphereBvhNode nd = root;
            if (b > 0) {
                for (int k = 0; k < 3; k++) {
                    const float lo = root.bmin[k], hi = root.bmax[k];
                    float x = lo + (float)u01(rng) * (hi - lo), y = lo + (float)u01(rng) * (hi - lo);
                    if (x > y) std::swap(x, y);
                    if (b % 7 == 1) x = std::nextafter(0.0f, 1.0f) * (float)(1 + b);  // denormal-scale values
                    if (b % 11 == 2) { x = -0.0f; y = 0.0f; }
                    nd.bmin[k] = std::fmax(std::fmin(x, hi), lo);
                    nd.bmax[k] = std::fmin(std::fmax(y, nd.bmin[k]), hi);
                }
                nd.leaf = (b % 2) ? (uint32_t)(b * 977) | (3u << 24) : kSphereBvhInternal;
                nd.skip = (uint32_t)b + 5u;
            }
            uint32_t q[4];
            tri_qnode(nd, g, q);
            float lo[3], hi[3];
            tri_qnode_box(q, g, lo, hi);
            for (int k = 0; k < 3; k++) {
                if (!(lo[k] <= nd.bmin[k] && hi[k] >= nd.bmax[k])) {
                    printf("CONTAIN case %ld box %d axis %d: [%.9g %.9g] vs [%.9g %.9g]\n", c, b, k, lo[k], hi[k],
                           nd.bmin[k], nd.bmax[k]);
                    return 1;
                }
                const uint32_t ql = k == 0 ? (q[0] & 0xffffu) : k == 1 ? (q[0] >> 16) : (q[1] & 0xffffu);
                const double exact = (double)g.origin[k] + (double)ql * (double)g.scale[k];
                if ((double)lo[k] != exact) {
                    printf("INEXACT case %ld axis %d\n", c, k);
                    return 1;
                }
            }
            const bool is_leaf = (q[3] & 0x80000000u) != 0u;
            if (is_leaf != (nd.leaf != kSphereBvhInternal) ||
                (is_leaf ? (q[3] & 0xffffffu) != (nd.leaf & 0xffffffu) : q[3] != nd.skip)) {
                printf("LINK case %ld box %d\n", c, b);
                return 1;
            }
            boxes++;
        }
    }
    printf("ok %ld %ld\n", cases, boxes);
    return 0;
}
