"""Ablation copies of the product kernels, for the timing tools only (never built into libvitdec.so).

The product headers (gpu-accelerated-viterbi-decoder_amd/csrc/vd_kernel_tg.h, vd_kernel_pk.h) carry no
ablation code.  This script writes tools/build/abl/vd_kernel_tg.h and vd_kernel_pk.h: the same kernels with a
template argument ABL (a set of kAbl* bits, 0 = the product kernel) that removes components (traceback,
read-out, table build, table reads, input loads, fairness controller, the two LDS exchanges, output stores)
or stamps s_memrealtime per wave.  Outputs of ABL != 0 are wrong by design.  Each patch below is a
(product text, tools text) pair that must occur exactly once in the product header: when the product
kernel changes, the script fails and names the pair to update (tests/test_tools_abl.py runs it on the CPU).
Tools include "build/abl/vd_kernel_pk.h" (tools/Makefile runs this script first).
Usage: python3 tools/abl/gen_abl.py [out_dir] [product csrc dir]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd", "csrc")

ABL_BITS = '''constexpr int kLlr = 8;
// Component ablations (tools only, tools/abl/gen_abl.py; the outputs are wrong): the template argument ABL
// of vd_decode_tg / vd_decode_pk is a set of these bits, 0 = the product kernel.
constexpr int kAblNoTraceback = 1, kAblNoTabReads = 2, kAblNoReadout = 4, kAblNoTabBuild = 8, kAblNoLoads = 16,
              kAblClock = 32, kAblNoFair = 256;
// vd_decode_pk study: trace back but keep the words in a register (no output stores)
constexpr int kAblNoStores = 524288;
constexpr int kAblAcsOnly = kAblNoTraceback | kAblNoTabReads | kAblNoReadout | kAblNoTabBuild | kAblNoLoads;
constexpr int kAblNoLdsX = 2097152;  // vd_decode_pk: the two LDS-exchange stages as DPP stages (wrong outputs)
// vd_decode_pk fairness studies (tools/vd_pkclock): the controller at every other group head (round 5's form);
// the controller in every batch of a batched launch
constexpr int kAblFair2 = 4194304, kAblFairAll = 67108864;'''

TG = [
    ("constexpr int kLlr = 8;", ABL_BITS),
    ("template <int CH, int CORE, int OB>\n__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(8))) void vd_decode_tg(",
     "template <int CH, int CORE, int OB, int ABL = 0>\n__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(8))) void vd_decode_tg("),
    ("    if (geo.check && lane < 3 * kGuardWords) wlds[LL::guard(lane)] = kGuardPattern;\n\n    // per-lane LDS byte offset",
     "    if (geo.check && lane < 3 * kGuardWords) wlds[LL::guard(lane)] = kGuardPattern;\n"
     "    const uint64_t t_clk0 = (ABL & kAblClock) ? __builtin_amdgcn_s_memtime() : 0;\n"
     "    const uint64_t t_rt0 = (ABL & kAblClock) ? __builtin_amdgcn_s_memrealtime() : 0;\n\n    // per-lane LDS byte offset"),
    ("    fair.begin(batch + 1 < geo.nbatch ? nullptr : geo.fair, lane);\n    // fairness progress",
     "    if constexpr (!(ABL & kAblNoFair)) fair.begin(batch + 1 < geo.nbatch ? nullptr : geo.fair, lane);\n    // fairness progress"),
    ("        if constexpr ((r / 6) % 2 == 0) {\n            vp[r] = *(lptr)(tl + aK[K] + TT::row(r));\n        }",
     "        if constexpr (ABL & kAblNoTabReads) {\n        } else if constexpr ((r / 6) % 2 == 0) {\n            vp[r] = *(lptr)(tl + aK[K] + TT::row(r));\n        }"),
    ("            const f2v e = vp[RP];", "            const f2v e = (ABL & kAblNoTabReads) ? (f2v){(float)aK[K], 1.0f} : vp[RP];"),
    ("            if constexpr (i % J == J - 1) {\n                // field read-out: bits 1..J of the pattern",
     "            if constexpr (i % J == J - 1 && !(ABL & kAblNoReadout)) {\n                // field read-out: bits 1..J of the pattern"),
    ("            if ((uint32_t)lane < nw && kb + lane >= E) {", "            if (!(ABL & kAblNoTraceback) && (uint32_t)lane < nw && kb + lane >= E) {"),
    ("        if constexpr (S01) {\n            float s0, s1;", "        if constexpr (S01 && !(ABL & kAblNoTabBuild)) {\n            float s0, s1;"),
    ("        } else {\n            using ab_t = std::conditional_t<IN::FAB, float, int>;",
     "        } else if constexpr (!(ABL & kAblNoTabBuild)) {\n            using ab_t = std::conditional_t<IN::FAB, float, int>;"),
    ("        {  // the next group's input words\n            rs = tg_rsrc<CH>(in, start + 32ull * (j + 3), availB);",
     "        if constexpr (!(ABL & kAblNoLoads)) {  // the next group's input words\n            rs = tg_rsrc<CH>(in, start + 32ull * (j + 3), availB);"),
    ("        if ((j / 3) % 2 == 0) fair.group((fdone + j) * fscale, 3u * fscale, lane);",
     "        if constexpr (!(ABL & kAblNoFair))\n            if ((j / 3) % 2 == 0) fair.group((fdone + j) * fscale, 3u * fscale, lane);"),
    ("    }  // pass\n    fair.end(lane);", "    }  // pass\n    if constexpr (!(ABL & kAblNoFair)) fair.end(lane);"),
    ("        if (lane == 0 && nbad) atomicAdd(geo.check, nbad);\n    }\n}\n\n}  // namespace vd",
     "        if (lane == 0 && nbad) atomicAdd(geo.check, nbad);\n    }\n"
     "    if constexpr (ABL & kAblClock) {\n"
     "        const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();\n"
     "        if (lane == 0) {\n"
     "            uint64_t* d = (uint64_t*)((char*)out + (16u << 20)) + 6 * (blockIdx.x * kWaves + wv);\n"
     "            d[0] = t_clk0; d[1] = c1; d[2] = t_rt0; d[3] = r1;\n"
     "            d[4] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));\n"
     "            d[5] = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11));\n"
     "        }\n    }\n}\n\n}  // namespace vd"),
]

PK = [
    ("// profiles/r05/ablate_nw7.log); 8 for batched HARD and SOFT4 (HARD loses 0.6-1.6 % at 7).\n"
     "template <int CH, int CORE, int OB = 32, bool SPL = false, int NW = (SPL || PkFmt<CH>::P2 || (CH & 7) == FP32) ? 7 : 8>\n",
     "// profiles/r05/ablate_nw7.log); 8 for batched HARD and SOFT4 (HARD loses 0.6-1.6 % at 7).  ABL: tools only\n"
     "// (component ablations as vd_decode_tg's, wrong outputs)\n"
     "template <int CH, int CORE, int OB = 32, bool SPL = false, int NW = (SPL || PkFmt<CH>::P2 || (CH & 7) == FP32) ? 7 : 8,\n"
     "          int ABL = 0>\n"),
    ("    const ChunkRange crA = chunk_range(geo, cA), crB = SPL ? crA : chunk_range(geo, cA + 1);\n",
     "    const ChunkRange crA = chunk_range(geo, cA), crB = SPL ? crA : chunk_range(geo, cA + 1);\n"
     "    // kAblClock (tools/vd_pkclock): s_memrealtime at the start, after the first pass and at the end\n"
     "    const uint64_t t_rt0 = (ABL & kAblClock) ? __builtin_amdgcn_s_memrealtime() : 0;\n"
     "    uint64_t t_rtp = 0;\n"
     "    uint32_t npass = 0;\n"),
    ("    fair.begin(batch + 1 < geo.nbatch ? nullptr : geo.fair, lane);",
     "    fair.begin(batch + 1 < geo.nbatch && !(ABL & kAblFairAll) ? nullptr : geo.fair, lane);"),
    ("    uint32_t cpv[kPkChk > 0 ? kPkChk : 1] = {};\n    uint32_t kb = 0;\n",
     "    uint32_t cpv[kPkChk > 0 ? kPkChk : 1] = {};\n    uint32_t kb = 0;\n    uint32_t sink = 0;  // kAblNoStores\n"),
    ("        if constexpr ((r / 6) % 2 == 0) vp[r] = *(lptr)(tl + aK[K] + TT::row(r));",
     "        if constexpr ((r / 6) % 2 == 0 && !(ABL & kAblNoTabReads)) vp[r] = *(lptr)(tl + aK[K] + TT::row(r));"),
    ("            const uint32_t m = ODD ? vp[RP].y : vp[RP].x;",
     "            const uint32_t m = (ABL & kAblNoTabReads) ? (uint32_t)aK[K] : ODD ? vp[RP].y : vp[RP].x;"),
    ("            if constexpr (Q <= 3) pk_stage_dpp<Q>(V, m);",
     "            if constexpr (Q <= 3 || (ABL & kAblNoLdsX)) pk_stage_dpp<(Q <= 3 ? Q : 0)>(V, m);"),
    ("            if constexpr (i % J == J - 1) {\n                // field read-out, both chunks",
     "            if constexpr (i % J == J - 1 && !(ABL & kAblNoReadout)) {\n                // field read-out, both chunks"),
    ("            if (tbl < nw && k >= (tbB ? kminB : kminA) && k < (tbB ? kmaxB : kmaxA)) {",
     "            if (!(ABL & kAblNoTraceback) && tbl < nw && k >= (tbB ? kminB : kminA) && k < (tbB ? kmaxB : kmaxA)) {"),
    ("                if constexpr (OB == 32) {\n                    ((uint32_t*)out)[tbStart + kc] = w;",
     "                if constexpr (ABL & kAblNoStores) {\n                    sink ^= w + kc;\n"
     "                } else if constexpr (OB == 32) {\n                    ((uint32_t*)out)[tbStart + kc] = w;"),
    ("            put_row(P0{}, rAA, rAB, sA, r6a);\n            if (lane < 32) put_row(P1{}, rBA, rBB, sB, r6b);\n",
     "            if constexpr (!(ABL & kAblNoTabBuild)) {\n                put_row(P0{}, rAA, rAB, sA, r6a);\n"
     "                if (lane < 32) put_row(P1{}, rBA, rBB, sB, r6b);\n            }\n"),
    ("            {  // the next group's input words\n                rsA = tg_rsrc<CH>(in, startA + 32ull * (j + 3), availB);",
     "            if constexpr (!(ABL & kAblNoLoads)) {  // the next group's input words\n                rsA = tg_rsrc<CH>(in, startA + 32ull * (j + 3), availB);"),
    ("            fair.group(j, 3u, lane);\n",
     "            if constexpr (!(ABL & kAblNoFair))\n                if (!(ABL & kAblFair2) || (j / 3) % 2 == 0) fair.group(j, 3u, lane);\n"),
    ("        if constexpr (!SPL) break;\n",
     "        if constexpr ((ABL & kAblClock) != 0) {\n            if (pass == 0) t_rtp = __builtin_amdgcn_s_memrealtime();\n"
     "            npass = pass + 1u;\n        }\n        if constexpr (!SPL) break;\n"),
    ("    fair.end(lane);\n    if (geo.check) {",
     "    fair.end(lane);\n"
     "    if constexpr ((ABL & kAblClock) != 0) {  // 8 words per wave behind the outputs (at least 16 MiB in)\n"
     "        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();\n"
     "        if (lane == 0) {\n"
     "            const uint64_t so = geo.nbatch * geo.outStride > (16u << 20) ? geo.nbatch * geo.outStride : (16u << 20);\n"
     "            uint64_t* d = (uint64_t*)((char*)out_all + so) + 8 * (blockIdx.x * kWaves + wv);\n"
     "            d[0] = t_rt0;\n"
     "            d[1] = t_rtp;\n"
     "            d[2] = t1;\n"
     "            d[3] = (uint32_t)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_ID\n"
     "            d[4] = (uint32_t)__builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11));  // XCC_ID\n"
     "            d[5] = npass;\n"
     "        }\n    }\n"
     "    if constexpr ((ABL & kAblNoStores) != 0) {\n"
     "        if (sink == 0x9E3779B9u) ((uint32_t*)out)[lane] = sink;  // keeps the traceback live\n"
     "    }\n    if (geo.check) {"),
]


def apply(text, patches, name, forward=True):
    for k, (prod, tools) in enumerate(patches):
        a, b = (prod, tools) if forward else (tools, prod)
        n = text.count(a)
        if n != 1:
            raise SystemExit(f"gen_abl.py: patch {k} of {name} matches {n} times (expected once); update it to the "
                             f"product header:\n{a[:300]}")
        text = text.replace(a, b)
    return text


def main(out_dir, csrc=CSRC):
    os.makedirs(out_dir, exist_ok=True)
    for name, patches in (("vd_kernel_tg.h", TG), ("vd_kernel_pk.h", PK)):
        src = open(os.path.join(csrc, name)).read()
        out = apply(src, patches, name)
        hdr = (f"// GENERATED by tools/abl/gen_abl.py from gpu-accelerated-viterbi-decoder_amd/csrc/{name}: the product\n"
               f"// kernel plus tools-only ablation bits (ABL).  Do not edit; never part of libvitdec.so.\n")
        with open(os.path.join(out_dir, name), "w") as f:
            f.write(hdr + out)


if __name__ == "__main__":
    # [out_dir] [csrc]: another product source tree (A/B of two kernel versions)
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tools", "build", "abl"),
         sys.argv[2] if len(sys.argv) > 2 else CSRC)
