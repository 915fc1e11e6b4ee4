// Microbenchmark: cycles per pop of the Kahn FIFO's single-successor step
// (topsort_lds, deg <= 1 branch) on one wave, over a chain of n nodes in LDS.
// Variants: (a) every lane writes the same LDS words (the current loop),
// (b) the three stores under lane 0 only, (c) only the node-word store,
// (d) no stores (read chain alone), (e) one store: queue entry when released,
// node word otherwise.  Output: cycles/pop.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kN = 8192;

template <int V>
__global__ void kpop(long long* out, int n)
{
    __shared__ uint32_t info[kN + 1];
    __shared__ uint16_t queue[kN + 1];
    __shared__ uint32_t qinfo[1024];
    const int lane = threadIdx.x;
    for (int v = lane; v < n; v += 64)
        info[v] = (v == 0 ? 0u : (1u << 24)) | (1u << 16) | uint32_t(v + 1 < n ? v + 1 : n);
    if (lane == 0)
        info[n] = 0xff000000u;
    __syncthreads();
    int tail       = 1;
    int q          = 0;
    uint32_t vinfo = __builtin_amdgcn_readfirstlane(info[0]);
    long long t0   = __builtin_amdgcn_s_memtime();
    while (q < tail)
    {
        tail  = __builtin_amdgcn_readfirstlane(tail);
        q     = __builtin_amdgcn_readfirstlane(q);
        vinfo = __builtin_amdgcn_readfirstlane(vinfo);
        const int deg     = int((vinfo >> 16) & 63u);
        const int o       = deg == 1 ? int(vinfo & 0xffffu) : n;
        const uint32_t oi = uint32_t(__builtin_amdgcn_readfirstlane(int(info[o]))) - (1u << 24);
        const bool rel    = deg == 1 && (oi >> 24) == 0u;
        if (V == 0)
        {
            info[o]                    = oi;
            queue[tail]                = uint16_t(o);
            qinfo[uint32_t(tail) & 1023] = oi;
        }
        else if (V == 1)
        {
            if (lane == 0)
            {
                info[o]                    = oi;
                queue[tail]                = uint16_t(o);
                qinfo[uint32_t(tail) & 1023] = oi;
            }
        }
        else if (V == 2)
            info[o] = oi;
        else if (V == 4)
        {
            // one store: the released node's queue entry, or the decremented word
            if (rel)
                queue[tail] = uint16_t(o);
            else
                info[o] = oi;
        }
        tail += rel ? 1 : 0;
        q++;
        vinfo = oi;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0)
    {
        out[0] = t1 - t0;
        out[1] = tail + queue[tail / 2] + qinfo[3];
    }
}

int main()
{
    long long* d;
    hipMalloc(&d, 1024 * 8);
    long long h[4];
    const int n = kN - 1;
    struct
    {
        const char* name;
        void (*k)(long long*, int);
    } ks[] = {{"all lanes store (current)", kpop<0>}, {"lane 0 stores", kpop<1>}, {"node word only", kpop<2>},
              {"no stores", kpop<3>},
              {"queue or word store", kpop<4>}};
    for (auto& k : ks)
    {
        hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, n);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, d, n);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("%-30s %.1f cycles/pop (check %lld)\n", k.name, double(h[0]) / n, h[1]);
    }
    return 0;
}
