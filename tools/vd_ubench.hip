// vd_ubench.hip -- gfx950 VALU issue-rate / latency microbenchmark for the ops the ACS loop uses.
// Throughput: 16 independent chains per wave, 8 waves/SIMD (grid 256 CUs x 32 waves).
// Latency: 1 dependent chain per wave, 1 wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define ITERS 2000

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

#define DEF_TP(NAME, INSTR)                                                                     \
__global__ void tp_##NAME(float* out, int n) {                                                  \
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,   \
          a6 = a0 + 6, a7 = a0 + 7, a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11,      \
          a12 = a0 + 12, a13 = a0 + 13, a14 = a0 + 14, a15 = a0 + 15;                           \
    float b = threadIdx.x * 0.5f;                                                               \
    for (int it = 0; it < n; it++) {                                                            \
        _Pragma("unroll") for (int u = 0; u < 4; u++) {                                        \
        asm volatile(                                                                           \
            INSTR("%0") INSTR("%1") INSTR("%2") INSTR("%3") INSTR("%4") INSTR("%5") INSTR("%6") INSTR("%7") \
            INSTR("%8") INSTR("%9") INSTR("%10") INSTR("%11") INSTR("%12") INSTR("%13") INSTR("%14") INSTR("%15") \
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),  \
              "+v"(a8), "+v"(a9), "+v"(a10), "+v"(a11), "+v"(a12), "+v"(a13), "+v"(a14), "+v"(a15) \
            : "v"(b) : "v40", "v41", "v42", "v43", "v44", "v45", "v50", "vcc");                  \
        }                                                                                       \
    }                                                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + a9 + a10 + a11 + a12 + a13 + a14 + a15; \
}                                                                                               \
__global__ void lat_##NAME(float* out, int n) {                                                 \
    float a0 = threadIdx.x; float b = threadIdx.x * 0.5f;                                       \
    for (int it = 0; it < n; it++) {                                                            \
        _Pragma("unroll") for (int u = 0; u < 4; u++) {                                        \
        asm volatile(INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") \
                     INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") INSTR("%0") \
                     : "+v"(a0) : "v"(b) : "v40", "v41", "v42", "v43", "v44", "v45", "v50", "vcc"); \
        }                                                                                       \
    }                                                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0;                                            \
}

// %16 is b in the tp kernels, %1 in lat kernels -> use a macro arg for the second operand
#define I_add_u32(d)      "v_add_u32 " d ", " d ", " d "\n"
#define I_add_f32(d)      "v_add_f32 " d ", " d ", " d "\n"
#define I_max_i32(d)      "v_max_i32 " d ", " d ", " d "\n"
#define I_max_f32(d)      "v_max_f32 " d ", " d ", " d "\n"
#define I_sub_u32_dpp(d)  "v_sub_u32_dpp " d ", " d ", " d " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define I_sub_f32_dpp(d)  "v_sub_f32_dpp " d ", " d ", " d " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define I_mov_dpp(d)      "v_mov_b32_dpp " d ", " d " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define I_pk_add_u16(d)   "v_pk_add_u16 " d ", " d ", " d "\n"
#define I_pk_max_i16(d)   "v_pk_max_i16 " d ", " d ", " d "\n"
#define I_pk_add_f16(d)   "v_pk_add_f16 " d ", " d ", " d "\n"
#define I_pk_max_f16(d)   "v_pk_max_f16 " d ", " d ", " d "\n"
#define I_alignbit(d)     "v_alignbit_b32 " d ", " d ", " d ", 31\n"
#define I_fma_f32(d)      "v_fma_f32 " d ", " d ", " d ", " d "\n"
#define I_sub_f32_clamp(d) "v_sub_f32 " d ", " d ", " d " clamp\n"
#define I_bfi(d)          "v_bfi_b32 " d ", " d ", " d ", " d "\n"
#define I_pk_lshr_b16(d)  "v_pk_lshrrev_b16 " d ", 1, " d "\n"
#define I_and_or(d)       "v_and_or_b32 " d ", " d ", " d ", " d "\n"
#define I_pk_fma_f32(d)   "v_pk_fma_f32 v[40:41], v[40:41], v[42:43], v[44:45]\n"
#define I_sub_u32(d)      "v_sub_u32 " d ", " d ", " d "\n"
#define I_lshl_add(d)     "v_lshl_add_u32 " d ", " d ", 1, " d "\n"
#define I_xor(d)          "v_xor_b32 " d ", " d ", " d "\n"
#define I_min_f32(d)      "v_min_f32 " d ", " d ", " d "\n"
#define I_add_i16(d)      "v_add_u16 " d ", " d ", " d "\n"
#define I_max3_f32(d)     "v_max3_f32 " d ", " d ", " d ", " d "\n"
#define I_med3_f32(d)     "v_med3_f32 " d ", " d ", " d ", " d "\n"
#define I_cvt_u32_f32(d)  "v_cvt_u32_f32 " d ", " d "\n"
#define I_permlane32(d)   "v_permlane32_swap_b32 " d ", v50\n"
#define I_swap_b32(d)     "v_swap_b32 " d ", v50\n"
#define I_bitop3(d)       "v_bitop3_b32 " d ", " d ", " d ", " d " bitop3:0x96\n"
#define I_pk_mul_f32(d)   "v_pk_mul_f32 v[40:41], v[40:41], v[42:43]\n"
#define I_add_co(d)       "v_add_co_u32 " d ", vcc, " d ", " d "\n"

#define LIST(X) X(add_u32) X(add_f32) X(max_i32) X(max_f32) X(sub_u32_dpp) X(sub_f32_dpp) X(mov_dpp) X(pk_add_u16) \
  X(pk_max_i16) X(pk_add_f16) X(pk_max_f16) X(alignbit) X(fma_f32) X(sub_f32_clamp) X(bfi) X(pk_lshr_b16) X(and_or) \
  X(pk_fma_f32) X(sub_u32) X(lshl_add) X(xor) X(min_f32) X(add_i16) X(max3_f32) X(med3_f32) X(cvt_u32_f32) \
  X(permlane32) X(bitop3) X(pk_mul_f32) X(add_co)

#define MK(N) DEF_TP(N, I_##N)
LIST(MK)

typedef void (*K)(float*, int);
struct E { const char* n; K tp; K lat; };
#define ENT(N) {#N, tp_##N, lat_##N},
static E ents[] = { LIST(ENT) };

int main() {
    float* out;
    CK(hipMalloc(&out, 256 * 32 * 64 * sizeof(float)));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    double ghz = clk / 1e6;
    printf("clock attr %.3f GHz\n", ghz);
    for (auto& e : ents) {
        float tp_ms = 0, lat_ms = 0;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0)); hipLaunchKernelGGL(e.tp, dim3(256 * 32), dim3(64), 0, 0, out, ITERS); CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&tp_ms, e0, e1));
            CK(hipEventRecord(e0)); hipLaunchKernelGGL(e.lat, dim3(256 * 4), dim3(64), 0, 0, out, ITERS); CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&lat_ms, e0, e1));
        }
        // tp: per SIMD: 8 waves x ITERS x 64 instr
        double tp_cyc = tp_ms * 1e-3 * 2.4e9 / (8.0 * ITERS * 64);
        double lat_cyc = lat_ms * 1e-3 * 2.4e9 / (1.0 * ITERS * 64);
        printf("%-16s throughput %.2f cyc/instr/SIMD   dep-latency %.2f cyc   (at 2.4 GHz)\n", e.n, tp_cyc, lat_cyc);
    }
    return 0;
}
