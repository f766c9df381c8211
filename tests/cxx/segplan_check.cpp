// Host check of the segment-launch geometry (vd_kernel_tg.h "segment launches", vd_segplan.h): for both
// tables and for many chunk-word patterns, the 4 segments of every workgroup cover each word of every
// chunk exactly once (emitted words), in order; every run starts at a chunk start (exact) or at a word
// a with (a + 1) % 3 == 0 and a >= the warm-up (3 and 6 blocks); every speculative start has a left neighbour ending at the
// same chunk block (its end vector is recorded at the block the start vector is); no segment is empty.
// Built with hipcc on the host by tests/test_segplan.py; prints "ok" or the first violation.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "vd_kernel_tg.h"
#include "vd_segplan.h"

using namespace vd;

static int fail(const char* what, int g, int q)
{
    printf("FAIL %s (workgroup %d, segment %d)\n", what, g, q);
    return 1;
}

static int check_table(const std::vector<uint32_t>& t, const std::vector<uint32_t>& words, uint32_t warm)
{
    for (size_t g = 0; g + 1 < t.size(); g++) {
        SegWG w;
        w.c0 = t[g];
        w.k = (int)(t[g + 1] - t[g]);
        w.warm = warm;
        if (w.k < 1 || w.k > kWaves) return fail("chunks per workgroup", (int)g, -1);
        uint32_t W[4] = {0, 0, 0, 0};
        for (int i = 0; i < w.k; i++) W[i] = words[w.c0 + i];
        w.W0 = W[0]; w.W1 = W[1]; w.W2 = W[2]; w.W3 = W[3];
        std::vector<std::vector<int>> cover(w.k);
        for (int i = 0; i < w.k; i++) cover[i].assign(W[i], 0);
        int endChunk[kWaves + 1], endBlock[kWaves + 1];  // where segment q's end vector is recorded
        for (int q = 0; q < kWaves; q++) {
            const SegPos b0 = seg_bound(w, q), b1 = seg_bound(w, q + 1);
            const int n = seg_nruns(b0, b1);
            if (n < 1) return fail("empty segment", (int)g, q);
            endChunk[q] = -1;
            for (int r = 0; r < n; r++) {
                const RunGeo rg = seg_run(w, b0, b1, r);
                if (rg.i < 0 || rg.i >= w.k) return fail("run chunk", (int)g, q);
                const uint32_t a = rg.s0 + rg.E, b = rg.s0 + rg.words;
                if (r > 0 && a != 0) return fail("later run not at a chunk start", (int)g, q);
                if (a > 0 && ((a + 1) % 3 != 0 || a < warm || rg.s0 % 3 != 0))
                    return fail("speculative start alignment", (int)g, q);
                if ((rg.Xspec >= 0) != (a > 0)) return fail("Xspec", (int)g, q);
                if (rg.Xspec >= 0 && (uint32_t)rg.Xspec + rg.s0 != a + 1) return fail("Xspec block", (int)g, q);
                if (b > W[rg.i] || a >= b) return fail("run range", (int)g, q);
                if ((rg.Xcmp >= 0) != (b < W[rg.i])) return fail("Xcmp", (int)g, q);
                if (rg.Xcmp >= 0 && ((uint32_t)rg.Xcmp + rg.s0 != b + 1 || r != n - 1)) return fail("Xcmp block", (int)g, q);
                if (rg.Xcmp >= 0) { endChunk[q] = rg.i; endBlock[q] = (int)(b + 1); }
                for (uint32_t k = a; k < b; k++) cover[rg.i][k]++;
                if (r == 0 && a > 0) {  // speculative start: the left neighbour ends at the same chunk block
                    if (q == 0 || endChunk[q - 1] != rg.i || endBlock[q - 1] != (int)(a + 1))
                        return fail("speculative start without a matching left end vector", (int)g, q);
                }
            }
        }
        for (int i = 0; i < w.k; i++)
            for (uint32_t k = 0; k < W[i]; k++)
                if (cover[i][k] != 1) return fail("word not covered exactly once", (int)g, i);
    }
    return 0;
}

// thirds / sevenths tables: each CU gets the intended mix of 4-chunk workgroups -- thirds: 1 of 8 (7 of 3
// chunks), sevenths: 4 of 7 (3 of 3 chunks) -- under both dealing orders of an XCD's workgroups to its 32
// CUs: round robin (CU n % 32) and per CU a run of consecutive n (CU n / per-CU count)
static int check_mix_per_cu(const std::vector<uint32_t>& t, int perCu, int wantFour, const char* name)
{
    const int nwg = (int)t.size() - 1, ncu = nwg / perCu;  // CUs of the chip (8 XCDs x 32)
    for (int order = 0; order < 2; order++) {
        std::vector<int> four(ncu), total(ncu);  // per (XCD, CU)
        for (int g = 0; g < nwg; g++) {
            const int x = g % 8, n = g / 8, cu = order == 0 ? n % 32 : n / perCu;
            total[x * 32 + cu]++;
            if (t[g + 1] - t[g] == 4) four[x * 32 + cu]++;
        }
        for (int c = 0; c < ncu; c++)
            if (four[c] != wantFour || total[c] != perCu) {
                printf("FAIL %s: CU %d gets %d 4-chunk workgroups of %d (dealing order %d)\n", name, c, four[c], total[c], order);
                return 1;
            }
    }
    return 0;
}

int main()
{
    int bad = 0;
    const int nsimd = 1024;  // 256 CUs
    bad |= check_mix_per_cu(seg_table(nsimd, kSegThirds), 8, 1, "thirds");
    bad |= check_mix_per_cu(seg_table(nsimd, kSegSevenths), 7, 4, "sevenths");
    for (int mode = 0; mode < 3; mode++) {
        const std::vector<uint32_t> t = seg_table(nsimd, mode);
        if (t.empty() || t.back() != (uint32_t)kChunks) { printf("FAIL table %d\n", mode); return 1; }
        // the bench sizes (32M and 16M bits, O_B32 and O_B16) and random word counts >= kSplitMinWords
        std::vector<uint32_t> packs = {999998, 499998, 1999996 / 2, 7999996 / 2};
        srand(7);
        for (int r = 0; r < 20; r++) packs.push_back(kChunks * (uint32_t)(kSplitMinWords + rand() % 400) + rand() % kChunks);
        for (uint32_t pack : packs) {
            std::vector<uint32_t> words(kChunks);
            for (uint32_t c = 0; c < (uint32_t)kChunks; c++) words[c] = pack / kChunks + (c < pack % kChunks ? 1 : 0);
            for (uint32_t warm : {3u, 6u}) bad |= check_table(t, words, warm);
        }
    }
    if (!bad) printf("ok\n");
    return bad;
}
