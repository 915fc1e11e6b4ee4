// Microbenchmark: cycles per loop iteration for a single wave with
// (a) straight-line scalar work, (b) the same work split by taken branches,
// (c) a dependent LDS read chain, (d) VALU chain.  Output: cycles/iteration.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void kstraight(long long* out, int n, int seed) {
    int x = seed;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        x = __builtin_amdgcn_readfirstlane(x);
#pragma unroll
        for (int k = 0; k < 10; k++) { x = x * 3 + k; x ^= (x >> 3); }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (t1 - t0); out[1] = x; }
}

__global__ void kbranchy(long long* out, int n, int seed) {
    int x = seed;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        x = __builtin_amdgcn_readfirstlane(x);
#pragma unroll
        for (int k = 0; k < 10; k++) {
            // data-dependent uniform branch: both sides do similar work
            if ((x >> k) & 1) { x = x * 3 + k; asm volatile("" : "+s"(x)); }
            else { x = x * 5 + k; asm volatile("" : "+s"(x)); }
            x ^= (x >> 3);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (t1 - t0); out[1] = x; }
}

__global__ void klds(long long* out, int n, int seed) {
    __shared__ int buf[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = (i * 7 + 1) & 1023;
    __syncthreads();
    int x = seed & 1023;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
        x = __builtin_amdgcn_readfirstlane(buf[x]);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (t1 - t0); out[1] = x; }
}

__global__ void kvalu(long long* out, int n, int seed) {
    int x = seed + threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 10; k++) x = x * 3 + k;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[2 + threadIdx.x] = x;
    if (threadIdx.x == 0) out[0] = (t1 - t0);
}

int main() {
    long long* d; hipMalloc(&d, 1024 * 8);
    long long h[4];
    const int n = 100000;
    struct { const char* name; void (*k)(long long*, int, int); int per; } ks[] = {
        {"straight (20 salu/iter)", kstraight, 1}, {"branchy (10 branches/iter)", kbranchy, 1},
        {"lds dependent chain", klds, 1}, {"valu dependent 10/iter", kvalu, 1}};
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, n, 12345);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, n, 12345);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("%-30s %.1f cycles/iter\n", k.name, double(h[0]) / n);
    }
    return 0;
}
