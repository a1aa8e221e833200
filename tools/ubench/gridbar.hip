// Grid-barrier cost on gfx950: G persistent workgroups, R barriers (atomic counter + generation,
// agent scope), against R back-to-back launches of an empty-ish kernel of the same grid.
// Build: hipcc -O3 --offload-arch=gfx950 gridbar.hip -o gridbar ; run: ./gridbar
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct Bar { unsigned count, gen; };

__device__ inline void grid_sync(Bar* b, unsigned nwg) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned g = __hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1) {
            __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&b->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(&b->gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

__global__ void k_bar(Bar* b, int rounds, double* buf) {
    double v = 0;
    for (int r = 0; r < rounds; r++) {
        buf[(blockIdx.x * blockDim.x + threadIdx.x)] += 1.0;  // some global traffic per phase
        grid_sync(b, gridDim.x);
        v += buf[((blockIdx.x + 1) % gridDim.x) * blockDim.x + threadIdx.x];
    }
    if (v < 0) buf[0] = v;
}

__global__ void k_one(const int* flag, double* buf) {
    if (*flag) return;
    buf[blockIdx.x * blockDim.x + threadIdx.x] += 1.0;
}

int main() {
    Bar* b; double* buf; int* flag;
    hipMalloc(&b, sizeof(Bar)); hipMemset(b, 0, sizeof(Bar));
    hipMalloc(&buf, 256 * 1024 * 8); hipMemset(buf, 0, 256 * 1024 * 8);
    hipMalloc(&flag, 4); hipMemset(flag, 0, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int R = 200;
    for (int threads : {256, 512}) {
        for (int G : {8, 16, 32, 64, 128, 256}) {
            float ms;
            hipLaunchKernelGGL(k_bar, dim3(G), dim3(threads), 0, 0, b, 10, buf);
            hipDeviceSynchronize();
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_bar, dim3(G), dim3(threads), 0, 0, b, R, buf);
            hipEventRecord(e1); hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            float ms2;
            hipEventRecord(e0);
            for (int r = 0; r < R; r++) hipLaunchKernelGGL(k_one, dim3(G), dim3(threads), 0, 0, flag, buf);
            hipEventRecord(e1); hipEventSynchronize(e1);
            hipEventElapsedTime(&ms2, e0, e1);
            printf("threads %d G %3d: grid barrier %.2f us, back-to-back launch %.2f us\n", threads, G, ms * 1e3 / R, ms2 * 1e3 / R);
        }
    }
    return 0;
}
