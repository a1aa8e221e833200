// Phase timing of k_octree (DistributeOctTree) on every level of image 0 of a real extraction
// (one workgroup traced per run: g_oct_trace_block; the launch numbers the levels from the top).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -DORBMI_OCT_TRACE \
//        -I include -I orb_slam2_with_comment_amd/csrc tools/octree_trace.hip \
//        orb_slam2_with_comment_amd/csrc/capi_extract.cpp orb_slam2_with_comment_amd/csrc/stereo.hip -o tools/octree_trace
// Run:   tools/octree_trace image.u8 rows cols [nfeatures]
#include "extractor.hip"

#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const int rows = atoi(argv[2]), cols = atoi(argv[3]);
    std::vector<uint8_t> img((size_t)rows * cols);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(img.data(), 1, img.size(), f) != img.size()) return 3;
    fclose(f);
    orbmi_extractor* h = nullptr;
    const int nf = argc > 4 ? atoi(argv[4]) : 2000, nl = 8;
    if (orbmi_extractor_create(0, nf, 1.2f, nl, 20, 7, &h)) return 4;
    std::vector<orbmi_keypoint> kps(16384);
    std::vector<uint8_t> desc(16384 * 32);
    int n = 0;
    for (int lv = 0; lv < nl; lv++) {
    const int blk = 8 * (nl - 1 - lv);  // image 0 of level lv (k_octree's numbering, one image)
    hipMemcpyToSymbol(HIP_SYMBOL(orbmi::g_oct_trace_block), &blk, sizeof(int));
    for (int it = 0; it < 5; it++)
        if (orbmi_extract(h, img.data(), rows, cols, cols, kps.data(), desc.data(), 16384, &n)) return 5;
    unsigned long long tr[256];
    hipMemcpyFromSymbol(tr, HIP_SYMBOL(orbmi::g_oct_trace), sizeof(tr));
    printf("== level %d: keypoints %d  keys %llu  iterations %llu  nodes %llu\n", lv, n, tr[62], tr[61], tr[60]);
    auto t = [&](int i) { return (long long)(tr[i] & ~(1ull << 63)); };
    printf("gather %lld  init %lld cycles\n", t(1) - t(0), t(2) - t(1));
    long long prev = t(2);
    for (int i = 0; i < (int)tr[61] && i < 50; i++) {
        printf("iter %2d%s %lld:", i, (tr[3 + i] >> 63) ? " (careful)" : "", t(3 + i) - prev);
        long long q = prev;
        for (int j = 0; j < 6 && i < 15; j++) { printf(" %lld", t(100 + 10 * i + j) - q); q = t(100 + 10 * i + j); }
        printf(" | %lld   [key pass: loads %lld atomics %lld spill %lld]\n", t(3 + i) - q, t(100 + 10 * i + 6) - t(100 + 10 * i),
               t(100 + 10 * i + 7) - t(100 + 10 * i + 6), t(100 + 10 * i + 8) - t(100 + 10 * i + 7));
        prev = t(3 + i);
    }
    printf("select+write %lld  total %lld cycles\n", t(59) - prev, t(59) - t(0));
    }
    orbmi_extractor_destroy(h);
    return 0;
}
