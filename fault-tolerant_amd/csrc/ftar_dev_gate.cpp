// ftar_dev_gate.cpp -- HIP runtime glue of libftar, part 3 of 4: launches queued ahead of
// their barrier behind a gate word (fdev_tree_batch_gated, fdev_run_gated), the gate's
// verdict, and the relaunch of a gated launch the device gave up (verify_gate).

#include <stdio.h>
#include <string.h>

#include "ftar_dev_impl.h"

using namespace fdevi;

namespace fdevi {

// Gate words: sig_flag[16 .. 23], gate `seq` in slot seq % kGateSlots; the slot's timeout
// word sig_flag[32 + slot] (a workgroup that gave the gate up writes the gate's value).
unsigned *gate_word(ftar_dev *d, unsigned seq) { return d->sig_flag + 16 + seq % ftar::kGateSlots; }
unsigned *gate_err(ftar_dev *d, unsigned seq) { return d->sig_flag + 32 + seq % ftar::kGateSlots; }

// Whether a launch of `grid` workgroups may be queued behind a gate now (see
// fdev_tree_batch_gated): a fenced marker or an unsignalled launch would have to drain
// behind the closed gate, a profiled launch would time the wait.
bool can_gate(const ftar_dev *d, unsigned grid)
{
    return d->flag_sync && !d->profiling && !d->gate_pending && !d->unsignalled && !d->force_fence && grid > 0 &&
           grid <= d->flag_max;
}

// The gate fields of a launch about to be queued gated; its bytes are counted when it runs.
ftar::KSignal arm_gate(ftar_dev *d, double link, double hbm)
{
    d->gate_link = link;
    d->gate_hbm = hbm;
    d->pre_gate_any = d->signalled > 0;
    d->pre_gate_tag = d->sig_tag;
    d->gate_seq++;
    d->signalled++;
    __atomic_store_n(gate_err(d, d->gate_seq), 0u, __ATOMIC_RELAXED); // the slot's last gate was verified
    // the workgroups invalidate their caches once the gate opens (acquire = 1): whatever
    // the drains before it did, the peers' data is read fresh
    ftar::KSignal k{};
    k.cnt = d->sig_cnt;
    k.flag = d->sig_flag;
    k.tag = ++d->sig_tag;
    k.acquire = d->tr_drop == 2 ? 0u : 1u; // tr_drop 2: TEST-ONLY
    k.gate = gate_word(d, d->gate_seq);
    k.gate_val = 2u * d->gate_seq;
    k.err = gate_err(d, d->gate_seq);
    k.gate_ticks = d->gate_ticks;
    return k;
}

// A short gated launch of several workgroups waits with ONE of them polling the host word
// over PCIe, the others polling the device word it relays the verdict through (the relayed
// form of the mid-size launches, signal_gate): up to 64 uncached PCIe pollers per launch
// slowed the peers sharing a GPU 2x at 1 MiB (RD, 4 ranks: 194 vs 93 us ungated).
void relay_gate(ftar_dev *d, ftar::KSignal &sig, unsigned grid)
{
    if (!d->gate_dw || grid < d->relay_min) return;
    sig.gate_poll = d->gate_dw + d->gate_seq % ftar::kGateSlots;
    sig.gate_dev = d->gate_dw + 32 + d->gate_seq % ftar::kGateSlots;
}

// Keep the plan of the gate just armed (d->gate_seq) for a relaunch: the same launch with
// no signal, gate or staging phase.
void keep_plan(ftar_dev *d, int batch, int dtype, int op, int nsrc, unsigned grid, const ftar::KSegList *L,
               const ftar::TreeBatch *B)
{
    ftar_dev::GatedPlan &g = d->gp[d->gate_seq & 1];
    g.valid = 1;
    g.opened = 0;
    g.batch = batch;
    g.dtype = dtype;
    g.op = op;
    g.nsrc = nsrc;
    g.grid = grid;
    g.seq = d->gate_seq;
    if (batch) {
        g.B = *B;
        g.B.sig = ftar::KSignal{};
    } else {
        g.L = *L;
        g.L.sig = ftar::KSignal{};
    }
}

} // namespace fdevi

extern "C" {

int fdev_tree_batch_staged_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                                 const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                                 void *stage_dst, const void *stage_src, size_t stage_n, int *gated)
{
    *gated = 0;
    if (!can_gate(d, 1)) return 0;
    ftar::TreeBatch B;
    unsigned grid = 0;
    double link, hbm;
    int rc = build_batch(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, &B, &grid, &link, &hbm);
    if (rc) return rc;
    // a one-shot of up to 4x the signal limit's workgroups still waits at its gate: its vector
    // workgroups take several chunks each (cap_tree_batch; the same tree per element)
    if (grid > d->flag_max && grid <= 4 * d->flag_max) {
        const unsigned g = ftar::cap_tree_batch(&B, d->flag_max);
        if (g) grid = g;
    }
    if (!can_gate(d, grid)) return 0;
    // only a launch that never writes what it reads is gated: a gate the device gave up on
    // is relaunched whole, and some workgroups may have run already
    const size_t es = esize_of(dtype);
    for (int t = 0; t < B.nt; t++)
        for (int k = 0; k < B.nt; k++)
            for (int j = 0; j < nsrc; j++)
                if (overlaps(B.t[t].out, B.t[t].n * es, B.t[k].src[j], B.t[k].n * es)) return 0;
    unsigned stage_tag = 0;
    if (stage_dst && stage_n) {
        stage_tag = ++d->sig_tag; // the launch raises the flag twice: staged, then done
        d->ctr.hbm_bytes += 2.0 * (double)stage_n * (double)es;
    }
    B.sig = arm_gate(d, link, hbm);
    relay_gate(d, B.sig, grid);
    keep_plan(d, 1, dtype, op, nsrc, grid, nullptr, &B);
    if (stage_tag) {
        B.sig.stage_src = stage_src;
        B.sig.stage_dst = stage_dst;
        B.sig.stage_n = stage_n;
        B.sig.stage_es = (unsigned)esize_of(dtype);
        B.sig.stage_tag = stage_tag;
        B.sig.stage_cnt = d->sig_cnt + 16; // its own counter, 64 B from the completion counter
        d->pre_gate_any = 1;               // the drain before the barrier waits for "staged"
        d->pre_gate_tag = stage_tag;
    }
    if (d->trace) {
        std::vector<TrRange> rd, wr, sw;
        batch_ranges(B, nsrc, es, rd, wr);
        const std::string rw = tr_rw(d, rd, wr);
        d->gp[d->gate_seq & 1].tr_rw = rw;
        std::string st;
        if (stage_tag) {
            sw.push_back({stage_dst, stage_n * es});
            tr_fmt(d, sw, st);
        }
        tr_launch(d, d->stream, &B.sig, rw, d->gate_seq, "k", st, stage_tag);
    }
    hipError_t e = ftar::launch_tree_batch(dtype, op, nsrc, B, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "tree_batch_kernel launch (gated)");
    d->gate_pending = 1;
    *gated = 1;
    return 0;
}

int fdev_tree_batch_gated(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc,
                          const unsigned *remote_mask, void *const *out, const size_t *n, int ntree, int tag,
                          int *gated)
{
    return fdev_tree_batch_staged_gated(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, nullptr, nullptr, 0,
                                        gated);
}

int fdev_gate_open(ftar_dev *d, int skip)
{
    if (!d->gate_pending) return 0;
    tr(d, "G %u %s", d->gate_seq, skip ? "skip" : "go");
    __atomic_store_n(gate_word(d, d->gate_seq), 2u * d->gate_seq + (skip ? 1u : 0u), __ATOMIC_RELEASE);
    if (!skip) {
        d->ctr.link_bytes += d->gate_link;
        d->ctr.hbm_bytes += d->gate_hbm;
    }
    d->gate_pending = 0;
    d->big_pending = 0;
    // a launch opened as go is checked at the drain that completes it (verify_gate); one given
    // up needs no check: its step launches normally, and the kept plan must never run after it
    ftar_dev::GatedPlan &g = d->gp[d->gate_seq & 1];
    if (g.valid && g.seq == d->gate_seq) {
        if (skip) g.valid = 0;
        else g.opened = 1;
    }
    return 0;
}

int fdev_gate_pending(const ftar_dev *d) { return d->gate_pending; }

int fdev_gate_relaunches(const ftar_dev *d) { return d->gate_relaunches; }

} // extern "C"

namespace fdevi {

// A mid-size launch (more workgroups than signal their completion cheaply) queued behind a
// gate: a fenced marker is recorded first -- the drain before the barrier waits for it, i.e.
// for everything queued before the gated launch, and its system-scope release makes that
// work visible to the peers as the usual drain does -- then the launch, its grid capped at
// big_blocks workgroups (each loops over its share of tiles: a waiting launch occupies a
// part of the device, so ranks sharing a GPU still run), its gate relayed through device
// words.  It does not signal: after the gate opens it is drained by a fenced marker.
int run_gated_relayed(ftar_dev *d, int dtype, int op, const ftar::SegIn *in, int nseg, size_t es, double link,
                      double hbm, int *gated)
{
    if (!d->flag_sync || !d->gate_dw || d->profiling || d->gate_pending) return 0;
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(in, nseg, es, d->big_blocks, &L);
    if (grid == 0) return 0;
    L.nt_store = nt_store();
    HIPCHK(hipEventRecord(d->fence_pre, d->stream)); // the work before the gate, released and drainable
    tr(d, "M pre");
    d->need_acquire = 0;
    L.sig = arm_gate(d, link, hbm);
    d->signalled--; // arm_gate counted a signalled launch: this one drains through a marker
    L.sig.cnt = nullptr;
    L.sig.flag = nullptr;
    L.sig.gate_poll = d->gate_dw + d->gate_seq % ftar::kGateSlots;
    L.sig.gate_dev = d->gate_dw + 32 + d->gate_seq % ftar::kGateSlots;
    keep_plan(d, 0, dtype, op, 0, grid, &L, nullptr);
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        for (int i = 0; i < nseg; i++) {
            rd.push_back({in[i].x, in[i].n * es});
            if (in[i].kind != ftar::kCopy) rd.push_back({in[i].y, in[i].n * es});
            wr.push_back({in[i].out, in[i].n * es});
            wr.push_back({in[i].out2, in[i].n * es});
        }
        const std::string rw = tr_rw(d, rd, wr);
        d->gp[d->gate_seq & 1].tr_rw = rw;
        d->tr_fenced = 0;
        tr_launch(d, d->stream, &L.sig, rw, d->gate_seq, "k");
    }
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch (gated, relayed)");
    d->gate_pending = 1;
    d->big_pending = 1;
    *gated = 1;
    return 0;
}

} // namespace fdevi

extern "C" {

int fdev_run_gated(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag, void *stage_dst,
                   const void *stage_src, size_t stage_n, int *gated)
{
    *gated = 0;
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || nseg < 0 || nseg > FDEV_MAX_SEGS || tag < 0 || tag >= FDEV_NTAGS) {
        snprintf(g_err, sizeof(g_err), "fdev_run_gated: bad arguments");
        return 13;
    }
    ftar::SegIn in[FDEV_MAX_SEGS];
    double link = 0, hbm = 0;
    seg_inputs(segs, nseg, es, in, &link, &hbm);
    // only a launch that never writes what it reads is gated (see fdev_tree_batch_staged_gated)
    for (int i = 0; i < nseg; i++)
        for (int k = 0; k < nseg; k++) {
            const size_t ni = segs[i].n * es, nk = segs[k].n * es;
            for (void *o : {segs[i].out, segs[i].out2})
                if (overlaps(o, ni, segs[k].x, nk) || (segs[k].kind != FDEV_COPY && overlaps(o, ni, segs[k].y, nk)))
                    return 0;
        }
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(in, nseg, es, d->max_blocks, &L);
    if (grid > d->flag_max && !stage_dst)
        return run_gated_relayed(d, dtype, op, in, nseg, es, link, hbm, gated);
    if (!can_gate(d, grid)) return 0;
    L.nt_store = nt_store();
    unsigned stage_tag = 0;
    if (stage_dst && stage_n) {
        stage_tag = ++d->sig_tag; // the launch raises the flag twice: staged, then done
        d->ctr.hbm_bytes += 2.0 * (double)stage_n * (double)es;
    }
    L.sig = arm_gate(d, link, hbm);
    relay_gate(d, L.sig, grid);
    keep_plan(d, 0, dtype, op, 0, grid, &L, nullptr);
    if (stage_tag) {
        L.sig.stage_src = stage_src;
        L.sig.stage_dst = stage_dst;
        L.sig.stage_n = stage_n;
        L.sig.stage_es = (unsigned)es;
        L.sig.stage_tag = stage_tag;
        L.sig.stage_cnt = d->sig_cnt + 16;
        d->pre_gate_any = 1;
        d->pre_gate_tag = stage_tag;
    }
    if (d->trace) {
        std::vector<TrRange> rd, wr, sw;
        seg_ranges(segs, nseg, es, rd, wr);
        const std::string rw = tr_rw(d, rd, wr);
        d->gp[d->gate_seq & 1].tr_rw = rw;
        std::string st;
        if (stage_tag) {
            sw.push_back({stage_dst, stage_n * es});
            tr_fmt(d, sw, st);
        }
        d->tr_fenced = 0;
        tr_launch(d, d->stream, &L.sig, rw, d->gate_seq, "k", st, stage_tag);
    }
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch (gated)");
    d->gate_pending = 1;
    *gated = 1;
    return 0;
}

} // extern "C"

namespace fdevi {

// The gates opened as go have completed (every drain covers the launches queued before any
// still-pending gate): did the device give one up (its gate stayed closed past the timeout,
// or a late workgroup found the slot overtaken)?  Then its workgroups (some or all) returned
// without touching memory, and the plan runs again ungated -- after a fenced marker
// (device-wide acquire: the peers' current data) and drained through one (release: visible
// to the peers before this rank arrives anywhere).  Any launch pending behind its own gate is
// given up first (nothing waits behind a closed gate); its step then launches normally.
int verify_gate(ftar_dev *d, int (*poll)(void *), void *arg)
{
    int redo = 0;
    for (unsigned k = 0; k < 2; k++) {
        // the older of the two first, and a later one again after a relaunch (it may have
        // read what the given-up one should have written): the steps' order is kept
        ftar_dev::GatedPlan &g = d->gp[(d->gate_seq + 1 + k) & 1];
        if (!g.valid || !g.opened) continue;
        g.valid = 0;
        unsigned *err = gate_err(d, g.seq);
        if (__atomic_load_n(err, __ATOMIC_ACQUIRE) != 2u * g.seq && !redo) continue;
        __atomic_store_n(err, 0u, __ATOMIC_RELAXED);
        if (d->gate_pending) (void)fdev_gate_open(d, 1);
        fprintf(stderr, "ftar: device %d: gated launch %u %s: relaunched\n", d->device, g.seq,
                redo++ ? "ran after a relaunched one" : "was given up by the device (gate timeout)");
        HIPCHK(hipEventRecord(d->fence_main, d->stream));
        d->tr_fenced = 1;
        tr_launch(d, d->stream, nullptr, g.tr_rw, 0, "k");
        hipError_t e = g.batch ? ftar::launch_tree_batch(g.dtype, g.op, g.nsrc, g.B, g.grid, d->stream)
                               : ftar::launch_segments(g.dtype, g.op, g.L, g.grid, d->stream);
        if (e != hipSuccess) return set_err(e, "relaunch of a timed-out gated launch");
        d->gate_relaunches++;
        int rc = sync_stream(d, d->stream, poll, arg);
        d->need_acquire = 0;
        d->unsignalled = d->signalled = d->force_fence = 0;
        if (rc) return rc;
    }
    return 0;
}

} // namespace fdevi
