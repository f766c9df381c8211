// vd_cuid.hip -- where the dispatcher puts the workgroups of a single-batch split launch (tools only): a kernel
// with the split kernel's footprint (256 threads, 20,480 B of LDS, 64 VGPRs, so 8 workgroups per CU fit)
// spins for a fixed number of cycles per workgroup and records its XCC / SE / CU from the hardware ID
// registers; prints workgroups per CU (histogram) for 1,600 workgroups (the split launch's 1,536 whole-chunk
// + 256 tail workgroups) and for other grid sizes.
// Usage: vd_cuid [spin cycles]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ __launch_bounds__(256) void spin(uint32_t* ids, uint64_t cycles)
{
    __shared__ uint32_t lds[5120];
    const uint64_t t0 = __builtin_readcyclecounter();
    uint32_t acc = threadIdx.x;
    while (__builtin_readcyclecounter() - t0 < cycles) {
        lds[threadIdx.x * 4 + (acc & 3)] = acc;
        acc = acc * 1664525u + 1013904223u;
    }
    if (threadIdx.x == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        ids[2 * blockIdx.x] = hw;
        ids[2 * blockIdx.x + 1] = xcc | (lds[acc & 1023] == 0x12345u ? 0x80000000u : 0u);
    }
}

int main(int argc, char** argv)
{
    const uint64_t cycles = argc > 1 ? strtoull(argv[1], nullptr, 10) : 200000;
    uint32_t* ids;
    CK(hipMalloc(&ids, 2 * 4 * 4096));
    for (int grid : {1600, 1792, 2048, 1536, 800}) {
        std::vector<uint32_t> h(2 * grid);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        hipLaunchKernelGGL(spin, dim3(grid), dim3(256), 0, 0, ids, cycles);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(spin, dim3(grid), dim3(256), 0, 0, ids, cycles);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(h.data(), ids, 8 * grid, hipMemcpyDeviceToHost));
        std::map<uint32_t, int> per_cu;
        for (int b = 0; b < grid; b++) {
            const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
            const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            per_cu[(xcc << 16) | (se << 8) | (sh << 4) | cu]++;
        }
        std::map<int, int> hist;
        for (auto& kv : per_cu) hist[kv.second]++;
        printf("grid %d: %.3f ms (spin %llu cycles), %zu CUs used; workgroups per CU:", grid, ms, (unsigned long long)cycles, per_cu.size());
        for (auto& kv : hist) printf(" %d x%d", kv.first, kv.second);
        printf("\n");
    }
    return 0;
}
