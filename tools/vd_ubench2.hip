// vd_ubench2.hip -- gfx950 VALU issue model for instruction MIXES (timing only).
// Each kernel body is an asm block repeated ITERS x 4 times; W waves per SIMD (grid 256 CUs x 4W waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define ITERS 1000

// registers: v[10:25] data, v26 = m, v27 = 2.0
#define PRO "v_mov_b32 v26, 1.0\n v_mov_b32 v27, 2.0\n"
#define CLOB "v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","vcc"

#define ADD(d) "v_add_f32 " d ", " d ", v26\n"
#define MAX(d) "v_max_f32 " d ", " d ", v26\n"
#define SUBDPP(d) "v_sub_f32_dpp " d ", " d ", v26 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define SUBCL(d) "v_sub_f32_e64 " d ", " d ", v26 clamp\n"
#define FMAC(d) "v_fmac_f32 " d ", 2.0, v26\n"

// one ACS stage for chain c: pm=v(10+c) t1=v(14+c) t2=v(18+c) bit=v(22+c) acc=v(30+c)
#define STAGE(P, T1, T2, BIT, ACC) \
    "v_add_f32 " T1 ", " P ", v26\n" \
    "v_sub_f32_dpp " T2 ", " P ", v26 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
    "v_max_f32 " P ", " T1 ", " T2 "\n" \
    "v_sub_f32_e64 " BIT ", " T1 ", " T2 " clamp\n" \
    "v_fmac_f32 " ACC ", 2.0, " BIT "\n"
#define STAGE_NODEC(P, T1, T2) \
    "v_add_f32 " T1 ", " P ", v26\n" \
    "v_sub_f32_dpp " T2 ", " P ", v26 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
    "v_max_f32 " P ", " T1 ", " T2 "\n"
#define STAGE_FMA(P, T1, T2, BIT, ACC) \
    "v_add_f32 " T1 ", " P ", v26\n" \
    "v_sub_f32_dpp " T2 ", " P ", v26 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n" \
    "v_sub_f32 " BIT ", " T1 ", " T2 "\n" \
    "v_max_f32 " P ", " T1 ", " T2 "\n" \
    "v_fma_f32 " ACC ", " ACC ", 2.0, " BIT " clamp\n"

#define K(NAME, BODY) \
__global__ void NAME(float* out, int n) { \
    float r = threadIdx.x; \
    asm volatile(PRO "v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, %0\n v_mov_b32 v13, %0\n v_mov_b32 v30, 0\n v_mov_b32 v31, 0\n v_mov_b32 v32, 0\n v_mov_b32 v33, 0\n" :: "v"(r) : CLOB); \
    for (int it = 0; it < n; it++) { asm volatile(BODY BODY BODY BODY ::: CLOB); } \
    asm volatile("v_add_f32 %0, v10, v30\n v_add_f32 %0, %0, v11\n v_add_f32 %0, %0, v31\n" : "=v"(r) :: CLOB); \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r; }

#define R16(M) M("v10") M("v11") M("v12") M("v13") M("v14") M("v15") M("v16") M("v17") M("v18") M("v19") M("v20") M("v21") M("v22") M("v23") M("v24") M("v25")
#define R8A(M) M("v10") M("v11") M("v12") M("v13") M("v14") M("v15") M("v16") M("v17")
#define R8B(M) M("v18") M("v19") M("v20") M("v21") M("v22") M("v23") M("v24") M("v25")
#define ALT8(A, B) A("v10") B("v18") A("v11") B("v19") A("v12") B("v20") A("v13") B("v21") A("v14") B("v22") A("v15") B("v23") A("v16") B("v24") A("v17") B("v25")

K(k_add16, R16(ADD))
K(k_max16, R16(MAX))
K(k_add8max8, ALT8(ADD, MAX))
K(k_dpp8add8, ALT8(SUBDPP, ADD))
K(k_dpp16, R16(SUBDPP))
K(k_subcl16, R16(SUBCL))
K(k_fmac16, R16(FMAC))
K(k_max8cl8, ALT8(MAX, SUBCL))
K(k_stage1, STAGE("v10", "v14", "v18", "v22", "v30") STAGE("v10", "v14", "v18", "v22", "v30") STAGE("v10", "v14", "v18", "v22", "v30") STAGE("v10", "v14", "v18", "v22", "v30"))
K(k_stage4, STAGE("v10", "v14", "v18", "v22", "v30") STAGE("v11", "v15", "v19", "v23", "v31") STAGE("v12", "v16", "v20", "v24", "v32") STAGE("v13", "v17", "v21", "v25", "v33"))
K(k_stage1_nodec, STAGE_NODEC("v10", "v14", "v18") STAGE_NODEC("v10", "v14", "v18") STAGE_NODEC("v10", "v14", "v18") STAGE_NODEC("v10", "v14", "v18"))
K(k_stage1_fma, STAGE_FMA("v10", "v14", "v18", "v22", "v30") STAGE_FMA("v10", "v14", "v18", "v22", "v30") STAGE_FMA("v10", "v14", "v18", "v22", "v30") STAGE_FMA("v10", "v14", "v18", "v22", "v30"))

struct E { const char* n; void (*k)(float*, int); int instrs_per_body; };

int main() {
    float* out; CK(hipMalloc(&out, 256 * 32 * 64 * sizeof(float)));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    E es[] = {{"add16", k_add16, 16}, {"max16", k_max16, 16}, {"add8max8", k_add8max8, 16}, {"dpp8add8", k_dpp8add8, 16},
              {"dpp16", k_dpp16, 16}, {"subclamp16", k_subcl16, 16}, {"fmac16", k_fmac16, 16}, {"max8subcl8", k_max8cl8, 16},
              {"stage x1 chain (5 ops)", k_stage1, 20}, {"stage x4 chains (5 ops)", k_stage4, 20},
              {"stage x1 nodec (3 ops)", k_stage1_nodec, 12}, {"stage x1 fma-clamp (5 ops)", k_stage1_fma, 20}};
    for (int W : {1, 2, 4, 7, 8}) {
        printf("--- %d waves/SIMD ---\n", W);
        for (auto& e : es) {
            std::vector<float> t;
            for (int r = 0; r < 5; r++) {
                CK(hipEventRecord(e0)); hipLaunchKernelGGL(e.k, dim3(256 * W), dim3(256), 0, 0, out, ITERS); CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            double ms = t[t.size() / 2];
            double per_body = ms * 1e-3 * 2.4e9 / (W * (double)ITERS * 4);  // SIMD cycles per body per wave
            printf("%-28s %8.2f cyc per body-per-wave  (%.2f cyc/instr/SIMD)\n", e.n, per_body, per_body / e.instrs_per_body);
        }
    }
    return 0;
}
