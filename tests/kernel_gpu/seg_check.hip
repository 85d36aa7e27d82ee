// TEST-ONLY: the product's segment kernel (every pull, copy, relay phase and guard store of
// the schedules) on its own, against the CPU oracle, bit for bit.
//
// Random segment lists as the schedules build them -- up to 16 pieces of copies and
// reduces, ragged lengths, element offsets that are co-aligned or not (vector body with
// scalar head / tail, or the scalar path), a second destination receiving the result again --
// planned by plan_segments at several grid caps (one tile per workgroup, and capped grids
// whose workgroups loop, as the mid-size gated launches run) and launched by
// launch_segments.  Expected values: copies as they are, reduces by the oracle's
// reduce_local (out = x op y, OpenMPI's operand roles), MAX / MIN over NaN, signed zeros and
// infinities.  Every byte around each destination is checked untouched.
//   seg_check [lists [swapped]]   prints one line per failing list, then "seg_check: N lists, F failed";
//   `swapped` expects y op x -- the checker's own test: float MAX / MIN lists must then fail
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

static void fill(unsigned char *buf, int dt, int op, size_t n, std::mt19937_64 &g)
{
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
            if (dt == ftar::kFloat32) {
                float f = (float)v;
                memcpy(buf + i * 4, &f, 4);
            } else {
                memcpy(buf + i * 8, &v, 8);
            }
        } else {
            const uint64_t v = r < 3 ? r : g();
            memcpy(buf + i * esize(dt), &v, esize(dt));
        }
    }
}

// one device allocation with a guard band around the operand
struct Buf {
    unsigned char *base = nullptr;
    size_t off = 0, bytes = 0;
    static constexpr size_t kPad = 64;
    void *ptr() const { return base + kPad + off; }
};

static Buf alloc(size_t bytes, size_t off, unsigned char fillbyte)
{
    Buf b;
    b.off = off;
    b.bytes = bytes;
    CHK(hipMalloc((void **)&b.base, bytes + 2 * Buf::kPad + 16));
    CHK(hipMemset(b.base, fillbyte, bytes + 2 * Buf::kPad + 16));
    return b;
}

int main(int argc, char **argv)
{
    const int lists = argc > 1 ? atoi(argv[1]) : 400;
    const bool swapped = argc > 2 && !strcmp(argv[2], "swapped");
    std::mt19937_64 g(4242);
    const int ops[][2] = {{ftar::kFloat32, ftar::kSum}, {ftar::kFloat32, ftar::kMax}, {ftar::kFloat32, ftar::kMin},
                          {ftar::kFloat64, ftar::kSum}, {ftar::kFloat64, ftar::kMin}, {ftar::kInt32, ftar::kSum},
                          {ftar::kInt32, ftar::kBor},   {ftar::kInt64, ftar::kProd}, {ftar::kInt64, ftar::kMax}};
    const unsigned caps[] = {1u << 20, 1024, 128, 7};
    int failed = 0;
    for (int li = 0; li < lists; li++) {
        const int *o = ops[li % (sizeof(ops) / sizeof(ops[0]))];
        const int dt = o[0], op = o[1];
        const size_t es = esize(dt);
        const unsigned cap = caps[(li / 9) % 4];
        const int nseg = 1 + (int)(g() % 16);
        const bool coalign = g() % 4 != 0;
        const size_t common = (size_t)(g() % 4) * es % 16;
        std::vector<ftar::SegIn> in(nseg);
        std::vector<Buf> outs, out2s, xs, ys;
        std::vector<std::vector<unsigned char>> hx(nseg), hy(nseg), want(nseg), want2(nseg);
        for (int s = 0; s < nseg; s++) {
            // mostly short pieces, some long ones (the interleaved prefix deals 128 KiB chunks)
            const size_t n = g() % 8 == 0 ? (size_t)(g() % (1u << 20)) + 1 : (size_t)(g() % 9000) + 1;
            auto off = [&]() { return coalign ? common : (size_t)(g() % 4) * es % 16; };
            const int kind = g() % 3 == 0 ? ftar::kCopy : ftar::kReduce;
            const bool with2 = g() % 3 != 0; // a second destination: the result again
            hx[s].resize(n * es);
            hy[s].resize(n * es);
            fill(hx[s].data(), dt, op, n, g);
            fill(hy[s].data(), dt, op, n, g);
            xs.push_back(alloc(n * es, off(), 0));
            ys.push_back(alloc(n * es, off(), 0));
            outs.push_back(alloc(n * es, off(), 0xA5));
            out2s.push_back(with2 ? alloc(n * es, off(), 0x5A) : Buf{});
            CHK(hipMemcpy(xs.back().ptr(), hx[s].data(), n * es, hipMemcpyHostToDevice));
            CHK(hipMemcpy(ys.back().ptr(), hy[s].data(), n * es, hipMemcpyHostToDevice));
            in[s].kind = kind;
            in[s].out = outs.back().ptr();
            in[s].x = xs.back().ptr();
            in[s].y = kind == ftar::kCopy ? nullptr : ys.back().ptr();
            in[s].n = n;
            in[s].out2 = with2 ? out2s.back().ptr() : nullptr;
            want[s] = swapped && kind == ftar::kReduce ? hy[s] : hx[s];
            if (kind == ftar::kReduce &&
                ftar_oracle_reduce_local(dt, op, (swapped ? hx[s] : hy[s]).data(), want[s].data(), n) != 0) {
                fprintf(stderr, "oracle refused dtype %d op %d\n", dt, op);
                return 2;
            }
            want2[s] = want[s];
        }
        ftar::KSegList L;
        const unsigned grid = ftar::plan_segments(in.data(), nseg, es, cap, &L);
        L.nt_store = (unsigned)(li & 1);
        memset(&L.sig, 0, sizeof(L.sig));
        bool ok = grid != 0;
        if (!ok) printf("FAIL list %d: plan_segments refused (%d pieces, cap %u)\n", li, nseg, cap);
        else CHK(ftar::launch_segments(dt, op, L, grid, 0));
        CHK(hipDeviceSynchronize());
        for (int s = 0; s < nseg && ok; s++) {
            const size_t n = in[s].n, bytes = n * es;
            for (int which = 0; which < 2 && ok; which++) {
                const Buf &b = which ? out2s[s] : outs[s];
                if (!b.base) continue;
                std::vector<unsigned char> whole(b.bytes + 2 * Buf::kPad + 16);
                CHK(hipMemcpy(whole.data(), b.base, whole.size(), hipMemcpyDeviceToHost));
                const std::vector<unsigned char> &w = which ? want2[s] : want[s];
                if (memcmp(whole.data() + Buf::kPad + b.off, w.data(), bytes)) {
                    size_t e = 0;
                    while (e < n && !memcmp(whole.data() + Buf::kPad + b.off + e * es, w.data() + e * es, es)) e++;
                    printf("FAIL list %d piece %d/%d (%s, n %zu, dtype %d op %d, cap %u, %s%s): element %zu\n", li, s,
                           nseg, in[s].kind == ftar::kCopy ? "copy" : "reduce", n, dt, op, cap,
                           which ? "second destination" : "out",
                           coalign ? ", co-aligned" : "", e);
                    ok = false;
                }
                const unsigned char fb = which ? 0x5A : 0xA5;
                for (size_t i = 0; i < whole.size() && ok; i++)
                    if ((i < Buf::kPad + b.off || i >= Buf::kPad + b.off + bytes) && whole[i] != fb) {
                        printf("FAIL list %d piece %d: byte %zu outside the destination written\n", li, s, i);
                        ok = false;
                    }
            }
            // the sources are never written
            std::vector<unsigned char> chk(bytes);
            CHK(hipMemcpy(chk.data(), xs[s].ptr(), bytes, hipMemcpyDeviceToHost));
            if (ok && chk != hx[s]) {
                printf("FAIL list %d piece %d: source x modified\n", li, s);
                ok = false;
            }
        }
        if (!ok) failed++;
        for (auto *v : {&outs, &out2s, &xs, &ys})
            for (auto &b : *v)
                if (b.base) CHK(hipFree(b.base));
    }
    printf("seg_check: %d lists, %d failed\n", lists, failed);
    return failed ? 1 : 0;
}
