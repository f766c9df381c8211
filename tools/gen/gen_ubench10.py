"""Generate tools/vd_ubench10.hip: gfx950 issue cost of single instructions and small mixes at 1/4/7
waves per SIMD, independent streams (16 rotating destination registers, no dependencies), plus the
tagged ACS stage as a dependent chain with 1 and 2 independent chains per wave.  Timing only."""
import sys

R = [f"v{10 + i}" for i in range(16)]
QP = "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
OPS = {
    "add": "v_add_f32 {d}, {d}, v40",
    "max": "v_max_f32 {d}, {d}, v40",
    "fma": "v_fma_f32 {d}, {d}, v40, v41",
    "dpp": "v_sub_f32_dpp {d}, {d}, v40 " + QP,
    "hmir": "v_sub_f32_dpp {d}, {d}, v40 row_half_mirror row_mask:0xf bank_mask:0xf",
    "ror8": "v_sub_f32_dpp {d}, {d}, v40 row_ror:8 row_mask:0xf bank_mask:0xf",
    "swap32": "v_permlane32_swap_b32 {d}, {e}",
    "swap16": "v_permlane16_swap_b32 {d}, {e}",
    "addu": "v_add_u32 {d}, {d}, v40",
    "and": "v_and_b32 {d}, {d}, v40",
    "bitop3": "v_bitop3_b32 {d}, {d}, v40, v41 bitop3:0x96",
    "nop": "s_nop 0",
    "pkadd": "v_pk_add_f32 v[{a}:{b}], v[{a}:{b}], v[40:41]",
    "dsread": "ds_read_b32 {d}, v42",
    "dsread64": "ds_read_b64 v[{a}:{b}], v42",
    "bpermute": "ds_bpermute_b32 {d}, v43, {d}",
}
SINGLE = ["add", "max", "fma", "dpp", "hmir", "ror8", "swap32", "swap16", "addu", "and", "bitop3", "nop", "pkadd",
          "dsread", "dsread64", "bpermute"]
MIX = [("add+max", ["add", "max"]), ("dpp+max", ["dpp", "max"]), ("add+dpp+max", ["add", "dpp", "max"]),
       ("add+nop+dpp+max", ["add", "nop", "dpp", "max"]), ("fma+fma+swap32+max", ["fma", "fma", "swap32", "max"]),
       ("add+dpp+max+dsread", ["add", "dpp", "max", "dsread"]), ("add+add+max+max", ["add", "add", "max", "max"])]


def inst(op, i):
    d = R[i % 16]
    e = R[(i + 1) % 16]
    a = 10 + 2 * (i % 8)
    return OPS[op].format(d=d, e=e, a=a, b=a + 1)


def body_single(op, n=32):
    return [inst(op, i) for i in range(n)]


def body_mix(ops, n=32):
    out = []
    for i in range(n // len(ops)):
        for j, op in enumerate(ops):
            out.append(inst(op, i * len(ops) + j))
    return out


def chain(nch, stages=24):
    """tagged DPP stage, nch independent chains interleaved"""
    out = []
    P = ["v10", "v11"]
    T1 = ["v14", "v15"]
    T2 = ["v18", "v19"]
    for s in range(stages):
        for c in range(nch):
            out.append(f"v_add_f32 {T1[c]}, {P[c]}, v40")
        out.append("s_nop 0")
        for c in range(nch):
            out.append(f"v_sub_f32_dpp {T2[c]}, {P[c]}, v40 {QP}")
        for c in range(nch):
            out.append(f"v_max_f32 {P[c]}, {T1[c]}, {T2[c]}")
    return out




def kstage(kind, P="v10", tab=False, nop_after=False):
    o = []
    if tab:
        o.append("ds_read_b32 v20, v42")
    if kind == "dpp":
        o += [f"v_add_f32 v14, {P}, v40", "s_nop 0", f"v_sub_f32_dpp v18, {P}, v40 {QP}", f"v_max_f32 {P}, v14, v18"]
    elif kind == "dpp_nonop":
        o += [f"v_add_f32 v14, {P}, v40", f"v_sub_f32_dpp v18, {P}, v40 {QP}", f"v_max_f32 {P}, v14, v18"]
    elif kind == "swapfma":
        o += [f"v_fma_f32 v14, v40, v41, {P}", f"v_fma_f32 v18, v40, -v41, {P}", "s_nop 1",
              "v_permlane32_swap_b32 v14, v18", f"v_max_f32 {P}, v14, v18"]
    elif kind == "swapadd":
        o += [f"v_add_f32 v14, {P}, v40", f"v_add_f32 v18, {P}, v41", "s_nop 1",
              "v_permlane32_swap_b32 v14, v18", f"v_max_f32 {P}, v14, v18"]
    elif kind == "swapadd_nonop":
        o += [f"v_add_f32 v14, {P}, v40", f"v_add_f32 v18, {P}, v41",
              "v_permlane32_swap_b32 v14, v18", f"v_max_f32 {P}, v14, v18"]
    elif kind == "swap_nop0":
        o += [f"v_fma_f32 v14, v40, v41, {P}", f"v_fma_f32 v18, v40, -v41, {P}", "s_nop 0",
              "v_permlane32_swap_b32 v14, v18", f"v_max_f32 {P}, v14, v18"]
    elif kind == "swap_mov":
        o += [f"v_mov_b32 v14, {P}", "s_nop 1", f"v_permlane32_swap_b32 v14, {P}",
              "v_add_f32 v18, v14, v40", f"v_sub_f32 v14, {P}, v40", f"v_max_f32 {P}, v14, v18"]
    elif kind == "swap_pk":
        o += [f"v_pk_add_f32 v[14:15], v[{P[1:]}:{int(P[1:])+1}], v[40:41] op_sel_hi:[0,1]", "s_nop 1",
              "v_permlane32_swap_b32 v14, v15", f"v_max_f32 {P}, v14, v15"]
    elif kind == "swap_max_nop":
        o += [f"v_fma_f32 v14, v40, v41, {P}", f"v_fma_f32 v18, v40, -v41, {P}", "s_nop 1",
              "v_permlane32_swap_b32 v14, v18", "s_nop 0", f"v_max_f32 {P}, v14, v18"]
    elif kind == "bperm":
        o += [f"ds_bpermute_b32 v18, v43, {P}", f"v_add_f32 v14, {P}, v40", "s_waitcnt lgkmcnt(0)",
              "v_sub_f32 v18, v18, v40", f"v_max_f32 {P}, v14, v18"]
    if tab:
        o.append("s_waitcnt lgkmcnt(0)")
    if nop_after:
        o.append("s_nop 0")
    return o


def seq(kinds, reps, **kw):
    out = []
    for _ in range(reps):
        for k in kinds:
            out += kstage(k, **kw)
    return out


PERIOD = ["swapfma", "dpp", "dpp", "dpp", "dpp", "swapfma"]
V = [(op, body_single(op), 32) for op in SINGLE] + [(n, body_mix(o), 32 // len(o) * len(o)) for n, o in MIX]
V += [("chain x1 (add,nop,dpp,max)/stage", chain(1), 24), ("chain x2 (2 chains)/stage-pair", chain(2), 24)]
V += [("K dpp stage", seq(["dpp"], 24), 24), ("K dpp stage, no nop", seq(["dpp_nonop"], 24), 24),
      ("K dpp stage + nop after", seq(["dpp"], 24, nop_after=True), 24),
      ("K swap stage (fma)", seq(["swapfma"], 24), 24), ("K swap stage (add)", seq(["swapadd"], 24), 24),
      ("K swap stage (add, no nop)", seq(["swapadd_nonop"], 24), 24), ("K bpermute stage", seq(["bperm"], 24), 24),
      ("K period 4dpp+2swap", seq(PERIOD, 4), 24), ("K period + nop after", seq(PERIOD, 4, nop_after=True), 24),
      ("K period + tab read", seq(PERIOD, 4, tab=True), 24),
      ("K swap stage nop0", seq(["swap_nop0"], 24), 24), ("K swap stage mov", seq(["swap_mov"], 24), 24),
      ("K swap stage pk_add", seq(["swap_pk"], 24, P="v12"), 24), ("K swap stage max-nop", seq(["swap_max_nop"], 24), 24)]
CLB = ','.join(f'"v{i}"' for i in list(range(10, 26)) + [40, 41, 42, 43])
src = ['// generated by tools/gen/gen_ubench10.py -- do not edit', '#include <hip/hip_runtime.h>', '#include <cstdio>',
       '#include <vector>', '#include <algorithm>',
       '#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\\n", hipGetErrorString(e)); return 1; } } while (0)']
ents = []
for i, (name, b, n) in enumerate(V):
    text = ''.join(s + '\\n' for s in b)
    wait = '"s_waitcnt lgkmcnt(0)\\n"' if any(x.startswith("ds_") for x in b) else '""'
    src.append(f'''__global__ __launch_bounds__(256) void k{i}(float* out, int n) {{
  __shared__ float lds[256];
  lds[threadIdx.x] = 1.0f;
  __syncthreads();
  float r = threadIdx.x;
  int bp = ((threadIdx.x & 63) ^ 32) * 4;
  asm volatile("v_mov_b32 v40, 1.0\\n v_mov_b32 v41, 2.0\\n v_mov_b32 v42, 0\\n v_mov_b32 v43, %1\\n"
    "v_mov_b32 v10, %0\\n v_mov_b32 v11, %0\\n v_mov_b32 v12, %0\\n v_mov_b32 v13, %0\\n v_mov_b32 v14, %0\\n v_mov_b32 v15, %0\\n v_mov_b32 v16, %0\\n v_mov_b32 v17, %0\\n"
    "v_mov_b32 v18, %0\\n v_mov_b32 v19, %0\\n v_mov_b32 v20, %0\\n v_mov_b32 v21, %0\\n v_mov_b32 v22, %0\\n v_mov_b32 v23, %0\\n v_mov_b32 v24, %0\\n v_mov_b32 v25, %0\\n" :: "v"(r), "v"(bp) : {CLB});
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; it++) {{ asm volatile("{text}" {wait} ::: {CLB}); }}
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  asm volatile("v_add_f32 %0, v10, v11\\n v_add_f32 %0, %0, v12\\n" : "=v"(r) :: {CLB});
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x == 0) ((unsigned long long*)out)[(1 << 20) + blockIdx.x] = c1 - c0; }}''')
    ents.append(f'{{"{name}", k{i}, {n}}}')
src.append('struct E { const char* n; void (*k)(float*, int); int per; };')
src.append('int main() { float* out; CK(hipMalloc(&out, 32u << 20)); hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));')
src.append('E es[] = {' + ','.join(ents) + '};')
src.append('''printf("%-36s %10s %10s %10s   (SIMD cycles per instruction-or-stage, per wave)\\n", "", "1 wave", "4 waves", "7 waves");
  for (auto& e : es) { printf("%-36s", e.n);
   for (int W : {1, 4, 7}) { std::vector<float> t; for (int r = 0; r < 4; r++) { CK(hipEventRecord(e0)); hipLaunchKernelGGL(e.k, dim3(256*W), dim3(256), 0, 0, out, 300); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r) t.push_back(ms); }
   std::vector<unsigned long long> c(256*W); CK(hipMemcpy(c.data(), (unsigned long long*)out + (1 << 20), 8*256*W, hipMemcpyDeviceToHost));
   std::sort(c.begin(), c.end()); double cyc = (double)c[c.size()/2]/(W*300.0*e.per);
   printf(" %10.2f", cyc); } printf("\\n"); }
 return 0; }''')
open(sys.argv[1], 'w').write('\n'.join(src) + '\n')
