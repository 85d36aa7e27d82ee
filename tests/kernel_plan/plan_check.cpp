// plan_check.cpp -- TEST: host-side coverage check of the segment kernel's work plan.
//
// For random multi-segment launches (1..16 segments, copy/reduce, 4- and 8-byte
// elements, co-aligned and misaligned pointers, sizes from 1 element to many chunks,
// capped and uncapped grids) it runs ftar::plan_segments and then walks every block of
// the grid through ftar::map_block -- the same function the kernel calls -- checking
// that every vector tile and every scalar element of every segment is processed
// exactly once and that the pieces tile the segments.  No GPU needed.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <vector>

#include "../../fault-tolerant_amd/csrc/ftar_kernels.h"

using namespace ftar;

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd()
{
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static int fail(const char *what, int c)
{
    fprintf(stderr, "case %d: %s\n", c, what);
    return 1;
}

int main(int argc, char **argv)
{
    int ncases = argc > 1 ? atoi(argv[1]) : 3000;
    int interleaved = 0, capped = 0;
    for (int c = 0; c < ncases; c++) {
        size_t es = (rnd() & 1) ? 4 : 8;
        int nin = 1 + (int)(rnd() % 16);
        SegIn in[16];
        for (int i = 0; i < nin; i++) {
            // disjoint fake address ranges; misalignment in element units
            uintptr_t base = ((uintptr_t)(i + 1) << 40);
            size_t mis_o = (rnd() % 4 == 0) ? (rnd() % (16 / es)) * es : 0;
            size_t mis_x = (rnd() % 8 == 0) ? (rnd() % (16 / es)) * es : mis_o;
            uint64_t r = rnd() % 10;
            size_t n = r < 2 ? 1 + rnd() % 300 : r < 6 ? 1 + rnd() % 200000 : 1 + rnd() % 3000000;
            in[i].kind = (rnd() & 1) ? kReduce : kCopy;
            in[i].out = (void *)(base + mis_o);
            in[i].x = (const void *)(base + ((uintptr_t)1 << 36) + mis_x);
            in[i].y = (const void *)(base + ((uintptr_t)2 << 36) + mis_o);
            in[i].n = n;
            in[i].out2 = (rnd() % 4 == 0) ? (void *)(base + ((uintptr_t)3 << 36) + mis_o) : nullptr;
        }
        unsigned max_blocks = (rnd() % 5 == 0) ? 64 + (unsigned)(rnd() % 2048) : 262144;
        KSegList L;
        unsigned grid = plan_segments(in, nin, es, max_blocks, &L);
        if (L.nil >= 2) interleaved++;
        if (max_blocks < 262144) capped++;
        // pieces tile their segments, with consistent operand offsets
        std::vector<std::vector<int>> cover_elem(L.nseg);
        for (int si = 0; si < L.nseg; si++) {
            const KSeg &S = L.s[si];
            int owner = -1;
            for (int i = 0; i < nin; i++) {
                intptr_t off = (intptr_t)S.out - (intptr_t)in[i].out;
                if (off >= 0 && (size_t)off < in[i].n * es) owner = i;
            }
            if (owner < 0) return fail("piece outside every segment", c);
            intptr_t off = (intptr_t)S.out - (intptr_t)in[owner].out;
            if ((intptr_t)S.x - (intptr_t)in[owner].x != off) return fail("x offset", c);
            if (in[owner].kind == kReduce && (intptr_t)S.y - (intptr_t)in[owner].y != off) return fail("y offset", c);
            if (S.vec && (((uintptr_t)S.out | (uintptr_t)S.x) & 15)) return fail("vector piece misaligned", c);
        }
        for (int i = 0; i < nin; i++) { // pieces of segment i cover [0, n) exactly once
            std::map<size_t, size_t> iv;
            for (int si = 0; si < L.nseg; si++) {
                intptr_t off = (intptr_t)L.s[si].out - (intptr_t)in[i].out;
                if (off >= 0 && (size_t)off < in[i].n * es) iv[(size_t)off / es] = L.s[si].n;
            }
            size_t at = 0;
            for (auto &kv : iv) {
                if (kv.first != at) return fail("pieces leave a gap or overlap", c);
                at += kv.second;
            }
            if (at != in[i].n) return fail("pieces do not cover the segment", c);
        }
        // every block's work: tiles / elements processed exactly once
        std::vector<std::vector<uint8_t>> seen(L.nseg);
        for (int si = 0; si < L.nseg; si++) {
            const KSeg &S = L.s[si];
            size_t units = S.vec ? (S.n / (16 / es) + kTileVecs - 1) / kTileVecs : (S.n + 255) / 256;
            seen[si].assign(units, 0);
        }
        for (unsigned b = 0; b < grid; b++) {
            BlockWork w = map_block(L, b);
            if (w.seg < 0 || w.seg >= L.nseg) return fail("block maps outside the list", c);
            if (w.stride == 0) return fail("zero stride", c);
            std::vector<uint8_t> &sv = seen[w.seg];
            for (size_t u = w.first; u < sv.size(); u += w.stride)
                if (++sv[u] > 1) return fail("unit processed twice", c);
        }
        for (int si = 0; si < L.nseg; si++)
            for (size_t u = 0; u < seen[si].size(); u++)
                if (seen[si][u] != 1) return fail("unit never processed", c);
    }
    printf("OK %d cases (%d interleaved, %d capped)\n", ncases, interleaved, capped);
    return (interleaved > 0 && capped > 0) ? 0 : 2;
}
