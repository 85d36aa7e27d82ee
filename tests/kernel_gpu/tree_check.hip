// TEST-ONLY: the mesh's tree kernels on their own, against the CPU oracle, bit for bit.
//
// tree_kernel<T, OP, P, U> (the one-hop mesh's reduce-scatter: the owner's block from p
// sources, the optional extra destinations of the push2 form) and tree_batch_kernel (the
// one-shot form: up to 8 trees in one launch) are launched directly -- every source a
// local buffer, so one process covers p = 2, 4, 8 AND 16 (the schedules only reach p = 16
// with 16 ranks, more GPU processes than a test may start beside its runner).  Expected
// values: the balanced left-to-right tree over the sources, each level computed by the
// oracle's reduce_local (oracle/ftar_oracle.c, OpenMPI's operand roles: inout op in), so
// the operand order of every combination is pinned (MAX / MIN over NaN, signed zeros and
// infinities).  Lengths ragged and co-aligned (vector body + scalar head / tail) or not
// (scalar path), unroll 1 / 2 / 4; batches also capped to 64 / 9 workgroups (cap_tree_batch:
// each vector workgroup loops over several chunks, as a gated one-shot launch runs).
//   tree_check [quick|swapped]   prints one line per failing case, then "tree_check: N cases, F failed";
//   `swapped` checks against the tree with every combination's operands swapped -- the
//   checker's own test: MAX / MIN cases must then fail
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "ftar_kernels.h"

extern "C" int ftar_oracle_reduce_local(int dtype, int op, const void *in, void *inout, size_t n);

#define CHK(x)                                                                                              \
    do {                                                                                                    \
        hipError_t e_ = (x);                                                                                \
        if (e_ != hipSuccess) {                                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));               \
            exit(2);                                                                                        \
        }                                                                                                   \
    } while (0)

static size_t esize(int dt) { return (dt == ftar::kInt64 || dt == ftar::kFloat64) ? 8 : 4; }

// random operands; MAX / MIN get NaNs, signed zeros and infinities (their results select an
// operand, so the order shows), SUM / PROD finite values and signed zeros only (IEEE leaves
// a NaN result's payload open, and the CPU and the GPU pick different defaults)
static void fill(std::vector<unsigned char> &buf, int dt, int op, size_t n, std::mt19937_64 &g)
{
    buf.resize(n * esize(dt));
    const bool sel = op == ftar::kMax || op == ftar::kMin;
    for (size_t i = 0; i < n; i++) {
        const unsigned r = (unsigned)(g() % 16);
        if (dt == ftar::kFloat32 || dt == ftar::kFloat64) {
            double v = std::ldexp((double)(int64_t)(g() % 2000001) - 1000000.0, -(int)(g() % 20));
            if (r == 0) v = 0.0;
            else if (r == 1) v = -0.0;
            else if (sel && r == 2) v = std::nan("");
            else if (sel && r == 3) v = -std::nan("");
            else if (sel && r == 4) v = INFINITY;
            else if (sel && r == 5) v = -INFINITY;
            if (op == ftar::kProd) v = (r & 1 ? 1.0 : -1.0) * (1.0 + (double)(g() % 8) / 1024.0);
            if (dt == ftar::kFloat32) {
                float f = (float)v;
                memcpy(&buf[i * 4], &f, 4);
            } else {
                memcpy(&buf[i * 8], &v, 8);
            }
        } else if (dt == ftar::kInt32) {
            uint32_t v = (uint32_t)g();
            if (r < 3) v = r; // zeros and ones for the logical ops
            memcpy(&buf[i * 4], &v, 4);
        } else {
            uint64_t v = g();
            if (r < 3) v = r;
            memcpy(&buf[i * 8], &v, 8);
        }
    }
}

// the balanced left-to-right tree over src[0..p-1], by the oracle
static bool g_swapped = false;

static std::vector<unsigned char> expect(const std::vector<std::vector<unsigned char>> &src, int p, int dt, int op,
                                         size_t n)
{
    std::vector<std::vector<unsigned char>> v(src.begin(), src.begin() + p);
    for (int w = 1; w < p; w *= 2)
        for (int j = 0; j < p; j += 2 * w) {
            const int a = g_swapped ? j + w : j, b = g_swapped ? j : j + w; // inout = inout op in
            if (ftar_oracle_reduce_local(dt, op, v[b].data(), v[a].data(), n) != 0) {
                fprintf(stderr, "oracle refused dtype %d op %d\n", dt, op);
                exit(2);
            }
            if (g_swapped) v[j] = v[j + w];
        }
    return v[0];
}

struct Case {
    int dt, op, p, unroll;
    size_t n;
    int misalign; // 0: every pointer 16-byte co-aligned at an element offset; 1: sources mutually misaligned
    int nmore;
};

static int g_fail = 0, g_cases = 0;

static void report(const char *what, const Case &c, const std::vector<unsigned char> &got,
                   const std::vector<unsigned char> &want)
{
    g_cases++;
    if (got == want) return;
    g_fail++;
    size_t es = esize(c.dt), first = 0;
    while (first < c.n && !memcmp(&got[first * es], &want[first * es], es)) first++;
    printf("FAIL %s dtype %d op %d p %d unroll %d n %zu misalign %d nmore %d: first difference at element %zu\n", what,
           c.dt, c.op, c.p, c.unroll, c.n, c.misalign, c.nmore, first);
}

static void run_tree(const Case &c, std::mt19937_64 &g)
{
    const size_t es = esize(c.dt), pad = 64, bytes = c.n * es;
    std::vector<std::vector<unsigned char>> src(c.p);
    for (int j = 0; j < c.p; j++) fill(src[j], c.dt, c.op, c.n, g);
    const std::vector<unsigned char> want = expect(src, c.p, c.dt, c.op, c.n);
    // one device arena per operand, the operand at an element offset inside it
    auto off = [&](int k) -> size_t {
        if (!c.misalign) return (size_t)(c.n % 3) * es % 16; // the same offset modulo 16 for every pointer
        return (size_t)(k % 4) * es % 16;                    // different offsets: no common vector body
    };
    std::vector<unsigned char *> arena(c.p + 1 + c.nmore);
    for (auto &a : arena) CHK(hipMalloc((void **)&a, bytes + pad));
    ftar::TreeArgs A;
    memset(&A, 0, sizeof(A));
    for (int j = 0; j < c.p; j++) {
        CHK(hipMemcpy(arena[j] + off(j), src[j].data(), bytes, hipMemcpyHostToDevice));
        A.src[j] = arena[j] + off(j);
    }
    A.out = arena[c.p] + off(c.p);
    CHK(hipMemset(arena[c.p], 0xA5, bytes + pad));
    for (int o = 0; o < c.nmore; o++) {
        A.more[o] = arena[c.p + 1 + o] + off(c.p + 1 + o);
        CHK(hipMemset(arena[c.p + 1 + o], 0x5A, bytes + pad));
    }
    A.nmore = c.nmore;
    A.n = c.n;
    A.unroll = (unsigned)c.unroll;
    A.nt_store = (unsigned)(c.n & 1);
    const unsigned grid = ftar::plan_tree(&A, c.p, es, 1u << 20);
    if (grid == 0) {
        printf("FAIL plan_tree refused p %d n %zu\n", c.p, c.n);
        g_fail++;
        return;
    }
    CHK(ftar::launch_tree(c.dt, c.op, c.p, A, grid, 0));
    CHK(hipDeviceSynchronize());
    std::vector<unsigned char> got(bytes), guard(pad);
    CHK(hipMemcpy(got.data(), A.out, bytes, hipMemcpyDeviceToHost));
    report("tree", c, got, want);
    // nothing written outside [out, out + n)
    std::vector<unsigned char> whole(bytes + pad);
    CHK(hipMemcpy(whole.data(), arena[c.p], bytes + pad, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < bytes + pad; i++)
        if ((i < off(c.p) || i >= off(c.p) + bytes) && whole[i] != 0xA5) {
            printf("FAIL tree wrote outside its block: p %d n %zu byte %zu\n", c.p, c.n, i);
            g_fail++;
            break;
        }
    for (int o = 0; o < c.nmore; o++) {
        CHK(hipMemcpy(got.data(), A.more[o], bytes, hipMemcpyDeviceToHost));
        report("tree (extra destination)", c, got, want);
    }
    for (auto a : arena) CHK(hipFree(a));
}

// the one-shot form: ntree trees of p sources each in one launch (tree k owns its workgroups)
static void run_batch(const Case &c, int ntree, std::mt19937_64 &g, unsigned cap = 0)
{
    const size_t es = esize(c.dt);
    ftar::TreeBatch B;
    memset(&B, 0, sizeof(B));
    B.nt = ntree;
    std::vector<std::vector<std::vector<unsigned char>>> src(ntree);
    std::vector<std::vector<unsigned char>> want(ntree);
    std::vector<unsigned char *> bufs;
    std::vector<size_t> ns(ntree);
    for (int k = 0; k < ntree; k++) {
        ns[k] = c.n + (size_t)k * 37; // ragged trees
        src[k].resize(c.p);
        for (int j = 0; j < c.p; j++) fill(src[k][j], c.dt, c.op, ns[k], g);
        want[k] = expect(src[k], c.p, c.dt, c.op, ns[k]);
        for (int j = 0; j < c.p; j++) {
            unsigned char *d;
            CHK(hipMalloc((void **)&d, ns[k] * es + 64));
            CHK(hipMemcpy(d, src[k][j].data(), ns[k] * es, hipMemcpyHostToDevice));
            B.t[k].src[j] = d;
            bufs.push_back(d);
        }
        unsigned char *o;
        CHK(hipMalloc((void **)&o, ns[k] * es + 64));
        B.t[k].out = o;
        B.t[k].n = ns[k];
        B.t[k].unroll = 1;
        bufs.push_back(o);
    }
    unsigned grid = ftar::plan_tree_batch(&B, c.p, es, 1u << 20);
    if (grid && cap && grid > cap) { // the gated one-shot's capped grid: vector workgroups loop
        const unsigned gc = ftar::cap_tree_batch(&B, cap);
        if (gc) grid = gc;
    }
    if (grid == 0) {
        printf("FAIL plan_tree_batch refused p %d n %zu\n", c.p, c.n);
        g_fail++;
    } else {
        CHK(ftar::launch_tree_batch(c.dt, c.op, c.p, B, grid, 0));
        CHK(hipDeviceSynchronize());
        for (int k = 0; k < ntree; k++) {
            std::vector<unsigned char> got(ns[k] * es);
            CHK(hipMemcpy(got.data(), B.t[k].out, got.size(), hipMemcpyDeviceToHost));
            Case ck = c;
            ck.n = ns[k];
            report("tree_batch", ck, got, want[k]);
        }
    }
    for (auto b : bufs) CHK(hipFree(b));
}

int main(int argc, char **argv)
{
    const bool quick = argc > 1 && (!strcmp(argv[1], "quick") || !strcmp(argv[1], "swapped"));
    g_swapped = argc > 1 && !strcmp(argv[1], "swapped");
    std::mt19937_64 g(20261017);
    const int ops[][2] = {{ftar::kFloat32, ftar::kSum}, {ftar::kFloat32, ftar::kMax}, {ftar::kFloat32, ftar::kMin},
                          {ftar::kFloat32, ftar::kProd}, {ftar::kFloat64, ftar::kSum}, {ftar::kFloat64, ftar::kMax},
                          {ftar::kInt32, ftar::kSum}, {ftar::kInt32, ftar::kLand}, {ftar::kInt64, ftar::kBxor},
                          {ftar::kInt64, ftar::kMin}};
    const size_t lens[] = {1, 3, 257, 4099, (1u << 16) + 5, (1u << 20) + 7};
    for (auto &o : ops)
        for (int p : {2, 4, 8, 16})
            for (int u : {1, 2, 4}) {
                if (u > 1 && p != 4 && p != 8) continue; // unrolled forms exist at p = 4, 8 only
                for (size_t n : lens) {
                    if (quick && n > 5000) continue;
                    if (n > 5000 && u > 1 && o[0] != ftar::kFloat32) continue; // keep the run short
                    for (int mis : {0, 1}) {
                        if (mis && n > 5000) continue; // the scalar path: short lengths suffice
                        const int nmore = (p <= 8 && n % 2) ? 2 : 0;
                        run_tree(Case{o[0], o[1], p, u, n, mis, nmore}, g);
                    }
                }
            }
    for (auto &o : ops)
        for (int p : {2, 4, 8})
            for (size_t n : {(size_t)5, (size_t)4099, (size_t)(1u << 16) + 3})
                for (int nt : {1, 3, 8})
                    for (unsigned cap : {0u, 64u, 9u})
                        run_batch(Case{o[0], o[1], p, 1, n, 0, 0}, nt, g, cap);
    printf("tree_check: %d cases, %d failed\n", g_cases, g_fail);
    return g_fail ? 1 : 0;
}
