"""Generate tools/vd_ubench12.hip: issue cost of the ACS building blocks at 7 waves per SIMD (single ops
on 16 independent registers: throughput) and of one-chain stage forms (the dependency chain one wave
carries through V).  Wall time from HIP events, ns per unit per SIMD.  Timing only (tools, not product)."""
import sys

QP = "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
R = [f"v{10 + i}" for i in range(16)]
OPS = {"add_f32": "v_add_f32 {d}, {d}, v40", "sub_f32": "v_sub_f32 {d}, {d}, v40",
       "max_f32": "v_max_f32 {d}, {d}, v40", "sub_f32_dpp": "v_sub_f32_dpp {d}, {d}, v40 " + QP,
       "max_f32_dpp": "v_max_f32_dpp {d}, {d}, v40 " + QP, "add_f32_dpp": "v_add_f32_dpp {d}, {d}, v40 " + QP,
       "mov_b32_dpp": "v_mov_b32_dpp {d}, {d} " + QP, "fma_f32": "v_fma_f32 {d}, {d}, v40, v41",
       "add_u32": "v_add_u32 {d}, {d}, v40", "max_i32": "v_max_i32 {d}, {d}, v40",
       "max_i32_dpp": "v_max_i32_dpp {d}, {d}, v40 " + QP, "sub_u32_dpp": "v_sub_u32_dpp {d}, {d}, v40 " + QP,
       "and_or_b32": "v_and_or_b32 {d}, {d}, v40, v41",
       "lshr_sdwa": "v_lshrrev_b32_sdwa {d}, 1, {d} dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD",
       "bfe_u32": "v_bfe_u32 {d}, {d}, 1, 8", "cvt_f32_i32": "v_cvt_f32_i32 {d}, {d}",
       "add3_u32": "v_add3_u32 {d}, {d}, v40, v41", "pk_max_u16": "v_pk_max_u16 {d}, {d}, v40",
       "pk_max_i16": "v_pk_max_i16 {d}, {d}, v40", "pk_add_u16": "v_pk_add_u16 {d}, {d}, v40",
       # the packed kernels' other opcodes (vd_kernel_pk.h read-out, traceback, table build)
       "sub_u32": "v_sub_u32 {d}, {d}, v40", "and_b32": "v_and_b32 {d}, 0x60006, {d}",
       "xad_u32": "v_xad_u32 {d}, {d}, v40, v41", "lshl_or_b32": "v_lshl_or_b32 {d}, {d}, 3, v40",
       "or3_b32": "v_or3_b32 {d}, {d}, v40, v41", "xor_b32": "v_xor_b32 {d}, {d}, v40",
       "lshlrev_b32": "v_lshlrev_b32 {d}, 3, {d}", "lshrrev_b32": "v_lshrrev_b32 {d}, 3, {d}",
       "bitop3_b32": "v_bitop3_b32 {d}, {d}, v40, v41 bitop3:0x96", "lshl_add_u32": "v_lshl_add_u32 {d}, {d}, 3, v40",
       "bfi_b32": "v_bfi_b32 {d}, v40, {d}, v41", "perm_b32": "v_perm_b32 {d}, {d}, v40, v41",
       "mul_u32_u24": "v_mul_u32_u24 {d}, {d}, v40", "cndmask_b32": "v_cndmask_b32 {d}, {d}, v40, vcc",
       "readfirstlane": "v_readfirstlane_b32 s20, {d}"}
PK = {"pk_add_f32": "v_pk_add_f32 v[{a}:{b}], v[{a}:{b}], v[40:41]",
      "pk_fma_f32": "v_pk_fma_f32 v[{a}:{b}], v[{a}:{b}], v[40:41], v[40:41]",
      "permlane32_swap": "v_permlane32_swap_b32 v{a}, v{b}", "permlane16_swap": "v_permlane16_swap_b32 v{a}, v{b}"}


def stage(kind, nch=1, stages=24):
    out = []
    for _ in range(stages):
        for c in range(nch):
            V, t1, t2 = f"v{10 + 4 * c}", f"v{11 + 4 * c}", f"v{12 + 4 * c}"
            if kind == "3op f32":
                out += [f"v_add_f32 {t1}, {V}, v40", "s_nop 0", f"v_sub_f32_dpp {t2}, {V}, v40 {QP}", f"v_max_f32 {V}, {t1}, {t2}"]
            elif kind == "2op f32":
                out += [f"v_sub_f32 {t2}, {V}, v40", f"v_add_f32 {t1}, {V}, v40", "s_nop 0", f"v_max_f32_dpp {V}, {t2}, {t1} {QP}"]
            elif kind == "3op i32":
                out += [f"v_add_u32 {t1}, {V}, v40", "s_nop 0", f"v_sub_u32_dpp {t2}, {V}, v40 {QP}", f"v_max_i32 {V}, {t1}, {t2}"]
            elif kind == "2op i32":
                out += [f"v_sub_u32 {t2}, {V}, v40", f"v_add_u32 {t1}, {V}, v40", "s_nop 0", f"v_max_i32_dpp {V}, {t2}, {t1} {QP}"]
            elif kind == "swap f32":
                a, b = 12 + 4 * c, 13 + 4 * c
                out += [f"v_pk_fma_f32 v[{a}:{b}], v[40:41], v[40:41], v[{10 + 4 * c}:{11 + 4 * c}] op_sel_hi:[1,1,0]",
                        "s_nop 1", f"v_permlane32_swap_b32 v{a}, v{b}", f"v_max_f32 {V}, v{a}, v{b}"]
            elif kind == "2op pk f32 (pair)":  # two states of one lane: pk add/sub, two max_dpp
                if c % 2: continue
                out += ["v_pk_add_f32 v[12:13], v[10:11], v[40:41]", "v_pk_add_f32 v[14:15], v[10:11], v[40:41] neg_lo:[0,1] neg_hi:[0,1]",
                        "s_nop 1", f"v_max_f32_dpp v10, v14, v12 {QP}", f"v_max_f32_dpp v11, v15, v13 {QP}"]
            elif kind == "3op pk f32 (pair)":  # pk add of the own candidates, two sub_dpp, two max
                if c % 2: continue
                out += ["v_pk_add_f32 v[12:13], v[10:11], v[40:41]", f"v_sub_f32_dpp v14, v10, v40 {QP}",
                        f"v_sub_f32_dpp v15, v11, v41 {QP}", "v_max_f32 v10, v12, v14", "v_max_f32 v11, v13, v15"]
            elif kind == "inlane pk (pair)":  # ps bit-5 stage: two pk_fma + two max
                if c % 2: continue
                out += ["v_pk_fma_f32 v[12:13], v[40:41], v[40:41], v[10:11] op_sel_hi:[1,1,0]",
                        "v_pk_fma_f32 v[14:15], v[40:41], v[40:41], v[10:11] op_sel:[0,0,1]",
                        "v_max_f32 v10, v12, v13", "v_max_f32 v11, v14, v15"]
            elif kind == "pk16 dpp (2 chunks)":  # mov_dpp of the packed pair, pk add / sub / max
                out += [f"v_mov_b32_dpp {t2}, {V} {QP}", f"v_pk_add_i16 {t1}, {V}, v40", f"v_pk_sub_i16 {t2}, {t2}, v40",
                        f"v_pk_max_i16 {V}, {t1}, {t2}"]
            elif kind == "pk16 plain (2 chunks)":  # partner value from elsewhere (LDS): pk add / sub / max
                out += [f"v_pk_add_i16 {t1}, {V}, v40", f"v_pk_sub_i16 {t2}, v41, v40", f"v_pk_max_i16 {V}, {t1}, {t2}"]
            elif kind == "pk32 dpp (2 chunks)":  # two int16 metrics per lane, 32-bit adds that never carry across
                out += [f"v_add3_u32 {t1}, {V}, v40, v41", "s_nop 0", f"v_sub_u32_dpp {t2}, {V}, v40 {QP}",
                        f"v_pk_max_u16 {V}, {t1}, {t2}"]
            elif kind == "pk32 plain (2 chunks)":  # partner value from elsewhere (LDS)
                out += [f"v_add3_u32 {t1}, {V}, v40, v41", f"v_sub_u32 {t2}, v41, v40", f"v_pk_max_u16 {V}, {t1}, {t2}"]
            elif kind == "pk32 dpp add (2 chunks)":  # cost reference: v_add_u32 in place of v_add3_u32
                out += [f"v_add_u32 {t1}, {V}, v40", "s_nop 0", f"v_sub_u32_dpp {t2}, {V}, v40 {QP}",
                        f"v_pk_max_u16 {V}, {t1}, {t2}"]
            elif kind == "add+max f32 (no exchange)":
                out += [f"v_add_f32 {t1}, {V}, v40", f"v_sub_f32 {t2}, {V}, v40", f"v_max_f32 {V}, {t1}, {t2}"]
    return out


V = [(op, [OPS[op].format(d=R[i % 16]) for i in range(32)], 32) for op in OPS]
V += [(op, [PK[op].format(a=10 + 2 * (i % 8), b=11 + 2 * (i % 8)) for i in range(32)], 32) for op in PK]
for k in ["3op f32", "2op f32", "3op i32", "2op i32", "swap f32", "add+max f32 (no exchange)"]:
    V.append((f"stage {k}", stage(k), 24))
    V.append((f"stage {k} x2 chains", stage(k, 2), 48))
for k in ["pk16 dpp (2 chunks)", "pk16 plain (2 chunks)", "pk32 dpp (2 chunks)", "pk32 plain (2 chunks)",
          "pk32 dpp add (2 chunks)"]:
    V.append((f"stage {k} per 2 states", stage(k), 24))
    V.append((f"stage {k} x2 chains per 2 states", stage(k, 2), 48))
for k in ["2op pk f32 (pair)", "3op pk f32 (pair)", "inlane pk (pair)"]:
    V.append((f"stage {k} per state", stage(k, 2), 48))
CLB = ','.join(f'"v{i}"' for i in list(range(10, 26)) + [40, 41]) + ', "vcc", "s20"'
src = ['// generated by tools/gen/gen_ubench12.py -- do not edit', '#include <hip/hip_runtime.h>', '#include <cstdio>',
       '#include <vector>', '#include <algorithm>',
       '#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\\n", hipGetErrorString(e)); return 1; } } while (0)']
ents = []
for i, (name, b, n) in enumerate(V):
    text = ''.join(s + '\\n' for s in b)
    movs = ''.join(f'v_mov_b32 v{r}, %0\\n' for r in range(10, 26))
    src.append(f'''__global__ __launch_bounds__(256) void k{i}(float* out, int n) {{
  float r = 12582912.0f + threadIdx.x;
  asm volatile("v_mov_b32 v40, 0x40400000\\n v_mov_b32 v41, 0x3f800000\\n{movs}" :: "v"(r) : {CLB});
  for (int it = 0; it < n; it++) {{ asm volatile("{text}" ::: {CLB}); }}
  asm volatile("v_add_f32 %0, v10, v11\\n" : "=v"(r) :: {CLB});
  out[blockIdx.x * blockDim.x + threadIdx.x] = r; }}''')
    ents.append(f'{{"{name}", k{i}, {n}}}')
src.append('struct E { const char* n; void (*k)(float*, int); int per; };')
src.append('int main(int argc, char** argv) { const int wps = argc > 1 ? atoi(argv[1]) : 7; float* out; CK(hipMalloc(&out, 64u << 20)); hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));')
src.append('E es[] = {' + ','.join(ents) + '};')
src.append('''printf("ns per unit per SIMD (wall), %d waves/SIMD\\n", wps);
  for (auto& e : es) { std::vector<float> t;
   for (int r = 0; r < 6; r++) { CK(hipEventRecord(e0)); hipLaunchKernelGGL(e.k, dim3(256*wps), dim3(256), 0, 0, out, 2000); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r) t.push_back(ms); }
   std::sort(t.begin(), t.end()); double ns = t[t.size()/2] * 1e6 / (wps * 2000.0 * e.per);
   printf("%-36s %8.3f ns\\n", e.n, ns); }
 return 0; }''')
open(sys.argv[1], 'w').write('\n'.join(src) + '\n')
