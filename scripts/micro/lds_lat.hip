// Micro-benchmark: cycles of one workgroup barrier, of a dependent LDS read
// chain, and of an independent batch of LDS reads (calibration for the
// level-keyed topological sort).  hipcc --offload-arch=gfx950 -O3 lds_lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void bench(unsigned long long* out, int iters)
{
    __shared__ unsigned int buf[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x)
        buf[i] = (i * 2654435761u + 12345u) & 4095u;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < iters; k++)
        __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned int x = threadIdx.x;
    for (int k = 0; k < iters; k++)
        x = buf[x & 4095u];
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    unsigned int y[8];
    for (int u = 0; u < 8; u++)
        y[u] = threadIdx.x + u * 64;
    for (int k = 0; k < iters; k++)
    {
#pragma unroll
        for (int u = 0; u < 8; u++)
            y[u] = buf[y[u] & 4095u];
    }
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
    unsigned int s = x;
    for (int u = 0; u < 8; u++)
        s += y[u];
    if (threadIdx.x == 0)
    {
        out[0] = (t1 - t0) / iters;
        out[1] = (t2 - t1) / iters;
        out[2] = (t3 - t2) / iters;
        out[3] = s;
    }
}

int main()
{
    unsigned long long* d;
    unsigned long long h[4];
    (void)hipMalloc(&d, 32);
    for (int threads : {64, 128, 256, 1024})
    {
        hipLaunchKernelGGL(bench, dim3(1), dim3(threads), 0, 0, d, 1000);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
        printf("threads %4d: barrier %llu cycles, dependent LDS read %llu cycles, 8 independent reads %llu cycles\n",
               threads, h[0], h[1], h[2]);
    }
    (void)hipFree(d);
    return 0;
}
