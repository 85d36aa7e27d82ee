// ftar_dev_trace.cpp -- HIP runtime glue of libftar, part 4 of 4: FTAR_TRACE, the per-rank
// log tests/fence_check.py checks (test instrumentation: nothing is written, and nothing
// costs anything, unless fdev_trace_open was called).

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ftar_dev_impl.h"

using namespace fdevi;

namespace fdevi {

// A launch's line: `L <n> s=<m|b> sig=<tag> rel=<0|1> acq=<0|1> fence=<0|1> gate=<seq> eng=<k|sdma>
// r=<regions read> w=<regions written> sw=<staged before the gate> stag=<tag>`, a region as
// owner:name:offset:bytes (only the registered ones: the workspaces, the exported send buffers and
// their peer mappings).  `rel` = the kernel releases its stores at system scope before it signals
// (signal_done), `acq` = it invalidates before its loads (signal_acquire), `fence` = a fenced marker
// was queued right in front of it.  tests/fence_check.py checks the cross-rank rules on the lines.
void tr(ftar_dev *d, const char *fmt, ...)
{
    if (!d->trace) return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(d->trace, fmt, ap);
    va_end(ap);
    fputc('\n', d->trace);
}

void tr_fmt(const ftar_dev *d, const std::vector<TrRange> &v, std::string &out)
{
    char buf[160];
    for (const TrRange &r : v) {
        if (!r.p || !r.n) continue;
        const uintptr_t a = (uintptr_t)r.p;
        for (const ftar_dev::Region &g : d->regions)
            if (a >= g.base && a < g.base + g.bytes) {
                snprintf(buf, sizeof(buf), "%d:%s:%zu:%zu,", g.owner, g.name.c_str(), (size_t)(a - g.base), r.n);
                out += buf;
                break;
            }
    }
    if (out.empty()) out = "-";
}

// The regions of a launch: "r=... w=..." (the relaunch of a gated plan reuses the text)
std::string tr_rw(const ftar_dev *d, const std::vector<TrRange> &rd, const std::vector<TrRange> &wr)
{
    if (!d->trace) return std::string();
    std::string a, b;
    tr_fmt(d, rd, a);
    tr_fmt(d, wr, b);
    return "r=" + a + " w=" + b;
}

void tr_launch(ftar_dev *d, hipStream_t st, const ftar::KSignal *sig, const std::string &rw, unsigned gate,
                      const char *eng, const std::string &staged, unsigned stag)
{
    if (!d->trace) return;
    const bool rel = sig && sig->cnt;
    const bool acq = sig && (sig->cnt || sig->gate) && sig->acquire;
    tr(d, "L %llu s=%c sig=%u rel=%d acq=%d fence=%d gate=%u eng=%s %s sw=%s stag=%u", ++d->tr_n,
       st == d->stream ? 'm' : 'b', rel ? sig->tag : 0u, rel ? 1 : 0, acq ? 1 : 0, d->tr_fenced, gate, eng, rw.c_str(),
       staged.empty() ? "-" : staged.c_str(), stag);
    d->tr_fenced = 0;
}

void seg_ranges(const fdev_seg *segs, int nseg, size_t es, std::vector<TrRange> &rd, std::vector<TrRange> &wr)
{
    for (int i = 0; i < nseg; i++) {
        const size_t b = segs[i].n * es;
        rd.push_back({segs[i].x, b});
        if (segs[i].kind != FDEV_COPY) rd.push_back({segs[i].y, b});
        wr.push_back({segs[i].out, b});
        wr.push_back({segs[i].out2, b});
    }
}

void batch_ranges(const ftar::TreeBatch &B, int nsrc, size_t es, std::vector<TrRange> &rd,
                  std::vector<TrRange> &wr)
{
    for (int t = 0; t < B.nt; t++) {
        for (int j = 0; j < nsrc; j++) rd.push_back({B.t[t].src[j], B.t[t].n * es});
        wr.push_back({B.t[t].out, B.t[t].n * es});
    }
}

} // namespace fdevi

extern "C" {

int fdev_trace_open(ftar_dev *d, const char *path)
{
    if (d->trace) return 0;
    d->trace = fopen(path, "w");
    if (!d->trace) {
        snprintf(g_err, sizeof(g_err), "FTAR_TRACE: cannot open %s", path);
        return 13;
    }
    setvbuf(d->trace, nullptr, _IOLBF, 0); // a killed rank leaves every line it wrote
#ifdef FTAR_TEST_HOOKS
    // TEST-ONLY (lib/libftar_hooks.so): drop a release or an acquire, so that
    // tests/test_gpu_fences.py can show the fence checker fails without it
    const char *dr = getenv("FTAR_TRACE_DROP");
    d->tr_drop = !dr ? 0 : !strcmp(dr, "release") ? 1 : !strcmp(dr, "acquire") ? 2 : 0;
#endif
    tr(d, "# ftar trace: device %d, flag_sync %d, drop %d", d->device, d->flag_sync, d->tr_drop);
    return 0;
}

void fdev_trace_region(ftar_dev *d, const void *base, size_t bytes, int owner, const char *name)
{
    if (!d->trace || !base) return;
    for (ftar_dev::Region &g : d->regions)
        if (g.base == (uintptr_t)base) {
            g.bytes = bytes;
            g.owner = owner;
            g.name = name;
            tr(d, "R %d %s %zu", owner, name, bytes);
            return;
        }
    d->regions.push_back(ftar_dev::Region{(uintptr_t)base, bytes, owner, name});
    tr(d, "R %d %s %zu", owner, name, bytes);
}

void fdev_trace_unregion(ftar_dev *d, const void *base)
{
    if (!d->trace || !base) return;
    for (size_t i = 0; i < d->regions.size(); i++)
        if (d->regions[i].base == (uintptr_t)base) {
            tr(d, "U %d %s", d->regions[i].owner, d->regions[i].name.c_str());
            d->regions.erase(d->regions.begin() + (long)i);
            return;
        }
}

// A write this rank's own launches did not make (the caller's send buffer, exported to the
// peers as it is): `X owner:name:offset:bytes`
void fdev_trace_external_write(ftar_dev *d, const void *p, size_t bytes)
{
    if (!d->trace) return;
    std::string w;
    tr_fmt(d, {{p, bytes}}, w);
    tr(d, "X %s", w.c_str());
}

void fdev_trace_note(ftar_dev *d, const char *fmt, ...)
{
    if (!d->trace) return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(d->trace, fmt, ap);
    va_end(ap);
    fputc('\n', d->trace);
}

} // extern "C"
