// Cost of back-to-back dependent kernel launches on one stream (no profiler): N launches of an
// empty kernel with G workgroups of B threads, timed with HIP events.  ./launch_cost
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;  // (vector store, never taken)
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int cfg[][2] = {{1, 64}, {1, 1024}, {94, 256}, {251, 512}, {1024, 256}};
    for (auto& c : cfg) {
        for (int rep = 0; rep < 2; rep++) {
            const int N = 2000;
            hipEventRecord(a, s);
            for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(c[0]), dim3(c[1]), 0, s, nullptr);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep) printf("grid %5d x %4d threads: %.2f us per launch\n", c[0], c[1], ms * 1e3 / N);
        }
    }
    // the same with an event record between launches (a marker packet per launch)
    hipEvent_t m;
    hipEventCreate(&m);
    const int N = 2000;
    hipEventRecord(a, s);
    for (int i = 0; i < N; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
        hipEventRecord(m, s);
    }
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    printf("1 x 64 + timed event record: %.2f us per launch\n", ms * 1e3 / N);
    hipEvent_t nt;
    hipEventCreateWithFlags(&nt, hipEventDisableTiming);
    hipEventRecord(a, s);
    for (int i = 0; i < N; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
        hipEventRecord(nt, s);
    }
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("1 x 64 + untimed event record: %.2f us per launch\n", ms * 1e3 / N);
    // cross-stream wait per launch (event recorded on a second stream, already complete)
    hipStream_t s2;
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEventRecord(nt, s2);
    hipStreamSynchronize(s2);
    hipEventRecord(a, s);
    for (int i = 0; i < N; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
        hipStreamWaitEvent(s, nt, 0);
    }
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    printf("1 x 64 + wait on a completed event of another stream: %.2f us per launch\n", ms * 1e3 / N);
    return 0;
}
