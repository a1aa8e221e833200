// FETCH_SIZE / WRITE_SIZE calibration on gfx950 (MI355X_MICROARCH.md §HBM: only 16-B-per-lane
// streaming reads are calibrated there).  Each kernel streams a 512 MiB buffer (past the 256 MiB
// Infinity Cache) once, coalesced, with 4-, 8- or 16-byte loads per lane, or writes it with
// stores of the same widths; run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`
// (separate passes) and compare the counters with the byte counts printed here.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/fetch_calib.hip -o tools/ubench/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBytes = 512ull << 20;

template <class V>
__global__ void k_read(const V* __restrict__ p, size_t n, unsigned* sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const V v = p[i];
        acc ^= (unsigned)reinterpret_cast<const unsigned*>(&v)[0];
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads
}

template <class V>
__global__ void k_write(V* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        V v;
        unsigned* w = reinterpret_cast<unsigned*>(&v);
        for (unsigned k = 0; k < sizeof(V) / 4; k++) w[k] = (unsigned)i + k;
        p[i] = v;
    }
}

int main() {
    unsigned char* buf;
    unsigned* sink;
    hipMalloc(&buf, kBytes);
    hipMalloc(&sink, 64);
    hipMemset(buf, 1, kBytes);
    const dim3 grid(4096), block(256);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_read<unsigned>, grid, block, 0, 0, (const unsigned*)buf, kBytes / 4, sink);
        hipLaunchKernelGGL(k_read<uint2>, grid, block, 0, 0, (const uint2*)buf, kBytes / 8, sink);
        hipLaunchKernelGGL(k_read<uint4>, grid, block, 0, 0, (const uint4*)buf, kBytes / 16, sink);
        hipLaunchKernelGGL(k_write<unsigned>, grid, block, 0, 0, (unsigned*)buf, kBytes / 4);
        hipLaunchKernelGGL(k_write<uint2>, grid, block, 0, 0, (uint2*)buf, kBytes / 8);
        hipLaunchKernelGGL(k_write<uint4>, grid, block, 0, 0, (uint4*)buf, kBytes / 16);
    }
    hipDeviceSynchronize();
    printf("every kernel moves %zu bytes (%.1f KiB): k_read<4/8/16 B>, k_write<4/8/16 B>\n", kBytes, kBytes / 1024.0);
    return 0;
}
