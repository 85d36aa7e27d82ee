// ftar_dev_launch.cpp -- HIP runtime glue of libftar, part 2 of 4: the launches of the
// segment and tree kernels and the copies on the rank's streams, their bookkeeping
// (completion signals, fenced markers), the drains (fdev_sync: a kernel's flag or a fenced
// marker), the device-ordered peer wait, and the host-buffer pipeline streams.

#include <stdio.h>
#include <string.h>

#include "ftar_dev_impl.h"

using namespace fdevi;

namespace fdevi {

// The background stream exists only in ranks that use it (Raben's step-0 redundancy
// copy with a spare): every stream is a hardware queue, and ranks that share a GPU (a
// spare beside its partner, the one-GPU test box) time-slice once the device's queue
// slots run out.
int ensure_bg(ftar_dev *d)
{
    if (d->bg) return 0;
    HIPCHK(hipStreamCreateWithFlags(&d->bg, hipStreamNonBlocking));
    // default (fenced) event: see sync_stream
    HIPCHK(hipEventCreateWithFlags(&d->fence_bg, hipEventDisableTiming));
    return 0;
}

hipEvent_t get_event(ftar_dev *d)
{
    if (!d->event_pool.empty()) {
        hipEvent_t e = d->event_pool.back();
        d->event_pool.pop_back();
        return e;
    }
    // pooled events only time kernels and order streams of this device: no system fence
    // (the cross-GPU visibility fence is sync_stream's dedicated marker)
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

// Bookkeeping of every launch or copy on a stream of this rank.  On the main stream: a
// launch of at most flag_max workgroups that may signal gets the completion signal
// (returned in *sig).  After a signal drain no marker packet has invalidated the caches
// (need_acquire): a signalled launch then invalidates them itself, per workgroup, for its
// own loads (`acquire`; an XCD's invalidate does nothing for the others, so need_acquire
// stays set), and any other launch is preceded by a fenced marker, which invalidates them
// device-wide as the drain's marker used to and clears need_acquire.  A background-stream
// launch gets such a marker on its own stream.
void note_launch(ftar_dev *d, hipStream_t st, unsigned grid, bool can_signal, ftar::KSignal *sig)
{
    if (sig) *sig = ftar::KSignal{};
    // anything queued behind a closed gate would wait for it: the gated launch is given up
    // (opened as skip; it returns untouched) -- its caller finds the gate no longer pending
    if (d->gate_pending) (void)fdev_gate_open(d, 1);
    d->tr_fenced = 0;
    const bool acquire = d->need_acquire && d->tr_drop != 2; // tr_drop 2: TEST-ONLY, acquires left out
    if (st != d->stream) {
        if (acquire && d->fence_bg) {
            (void)hipEventRecord(d->fence_bg, st);
            d->tr_fenced = 1;
        }
        return;
    }
    if (can_signal && sig && d->flag_sync && grid <= d->flag_max) {
        *sig = ftar::KSignal{};
        sig->cnt = d->sig_cnt;
        sig->flag = d->sig_flag;
        sig->tag = ++d->sig_tag;
        sig->acquire = (unsigned)acquire;
        d->signalled++;
    } else {
        if (acquire) {
            (void)hipEventRecord(d->fence_main, st);
            d->tr_fenced = 1;
        }
        d->need_acquire = 0;
        d->unsignalled++;
    }
}

// The kernel's view of fdev segments, and their algorithmic link / HBM bytes.
void seg_inputs(const fdev_seg *segs, int nseg, size_t es, ftar::SegIn *in, double *link, double *hbm)
{
    for (int i = 0; i < nseg; i++) {
        in[i].kind = segs[i].kind == FDEV_COPY ? ftar::kCopy : ftar::kReduce;
        in[i].out = segs[i].out;
        in[i].x = segs[i].x;
        in[i].y = segs[i].y;
        in[i].n = segs[i].n;
        in[i].out2 = segs[i].out2;
        double b = (double)segs[i].n * (double)es;
        int nread = segs[i].kind == FDEV_COPY ? 1 : 2;
        int nremote = ((segs[i].remote & FDEV_REMOTE_X) ? 1 : 0) +
                      ((segs[i].kind != FDEV_COPY && (segs[i].remote & FDEV_REMOTE_Y)) ? 1 : 0);
        int rout = (segs[i].remote & FDEV_REMOTE_OUT) ? 1 : 0;
        *link += b * (nremote + rout);
        *hbm += b * (1 - rout + nread - nremote + (segs[i].out2 ? 1 : 0));
    }
}

// [a, a + na) and [b, b + nb) overlap
bool overlaps(const void *a, size_t na, const void *b, size_t nb)
{
    const char *x = (const char *)a, *y = (const char *)b;
    return a && b && x < y + nb && y < x + na;
}

int run_on(ftar_dev *d, hipStream_t st, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || nseg < 0 || nseg > FDEV_MAX_SEGS || tag < 0 || tag >= FDEV_NTAGS) {
        snprintf(g_err, sizeof(g_err), "fdev_run: bad arguments");
        return 13;
    }
    ftar::SegIn in[FDEV_MAX_SEGS];
    double link = 0, hbm = 0;
    seg_inputs(segs, nseg, es, in, &link, &hbm);
    d->ctr.link_bytes += link;
    d->ctr.hbm_bytes += hbm;
    ftar::KSegList L;
    unsigned grid = ftar::plan_segments(in, nseg, es, d->max_blocks, &L);
    const bool behind_wait = d->pw_pending && st == d->stream;
    if (behind_wait) d->pw_pending = 0;
    if (grid == 0) return 0;
    L.nt_store = nt_store();
    note_launch(d, st, grid, true, &L.sig);
    if (behind_wait) {
        // behind a peer wait: the wait's verdict decides.  No acquire of its own: the fenced
        // marker in front of the flag (fdev_peer_wait) invalidated this GPU's caches after
        // everything this rank read before, and since then only the wait kernel has read
        // anything (the flag words, in host memory) -- no line of what this launch reads can
        // be stale (tests/fence_check.py's acquire rule checks exactly that on the logs)
        L.sig.vword = d->gate_dw + 48;
        L.sig.vval = d->pw_vval;
        d->pw_armed = 1;
    }
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        seg_ranges(segs, nseg, es, rd, wr);
        tr_launch(d, st, &L.sig, tr_rw(d, rd, wr), 0, "k");
        if (behind_wait) d->pw_launch_n = d->tr_n;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, st);
    }
    hipError_t e = ftar::launch_segments(dtype, op, L, grid, st);
    if (e != hipSuccess) return set_err(e, "segment_kernel launch");
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, st);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

} // namespace fdevi

extern "C" {

int fdev_tree(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
              size_t n, int tag)
{
    return fdev_tree_out(d, dtype, op, src, nsrc, remote_mask, out, nullptr, 0, 0, n, tag);
}

int fdev_tree_out(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, unsigned remote_mask, void *out,
                  void *const *more, int nmore, int more_remote, size_t n, int tag)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || tag < 0 || tag >= FDEV_NTAGS ||
        !(nsrc == 2 || nsrc == 4 || nsrc == 8 || nsrc == 16) || nmore < 0 || nmore > ftar::kMaxMore) {
        snprintf(g_err, sizeof(g_err), "fdev_tree: bad arguments");
        return 13;
    }
    if (n == 0) return 0;
    int nremote = __builtin_popcount(remote_mask & ((1u << nsrc) - 1));
    const int mr = more_remote ? nmore : 0; // extra destinations in peers' HBM, or in ours
    d->ctr.link_bytes += (double)n * (double)es * (nremote + mr);
    d->ctr.hbm_bytes += (double)n * (double)es * (nsrc - nremote + 1 + nmore - mr);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, d->stream);
    }
    note_launch(d, d->stream, ~0u, false, nullptr);
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        for (int j = 0; j < nsrc; j++) rd.push_back({src[j], n * es});
        wr.push_back({out, n * es});
        for (int o = 0; o < nmore; o++) wr.push_back({more[o], n * es});
        tr_launch(d, d->stream, nullptr, tr_rw(d, rd, wr), 0, "k");
    }
    // pieces of at most max_blocks vector workgroups (plan_tree refuses larger bodies)
    const unsigned u = (nsrc == 4 || nsrc == 8) ? d->tree_unroll : 1u;
    const size_t piece = (size_t)d->max_blocks * 256 * u * (16 / es);
    for (size_t off = 0; off < n; off += piece) {
        ftar::TreeArgs A;
        memset(&A, 0, sizeof(A));
        for (int j = 0; j < nsrc; j++) A.src[j] = (const char *)src[j] + off * es;
        A.out = (char *)out + off * es;
        A.nmore = nmore;
        for (int o = 0; o < nmore; o++) A.more[o] = (char *)more[o] + off * es;
        A.n = n - off < piece ? n - off : piece;
        A.nt_store = nt_store();
        A.unroll = u;
        unsigned grid = ftar::plan_tree(&A, nsrc, es, d->max_blocks + 1);
        if (grid == 0) {
            snprintf(g_err, sizeof(g_err), "fdev_tree: plan failed");
            return 13;
        }
        hipError_t e = ftar::launch_tree(dtype, op, nsrc, A, grid, d->stream);
        if (e != hipSuccess) return set_err(e, "tree_kernel launch");
    }
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, d->stream);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

} // extern "C"

namespace fdevi {

// The TreeBatch of fdev_tree_batch(_gated): the grid (0 = a tree beyond the workgroup
// budget, or nothing to do when B->nt == 0), link and HBM bytes.
int build_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                void *const *out, const size_t *n, int ntree, int tag, ftar::TreeBatch *B, unsigned *grid,
                double *link, double *hbm)
{
    size_t es = esize_of(dtype);
    if (es == 0 || op < 0 || op >= ftar::kNumOps || tag < 0 || tag >= FDEV_NTAGS || ntree < 1 || ntree > ftar::kMaxBatch ||
        !(nsrc == 2 || nsrc == 4 || nsrc == 8)) {
        snprintf(g_err, sizeof(g_err), "fdev_tree_batch: bad arguments");
        return 13;
    }
    memset(B, 0, sizeof(*B));
    B->nt = 0;
    *link = *hbm = 0;
    for (int t = 0; t < ntree; t++) {
        if (n[t] == 0) continue;
        ftar::TreeArgs &A = B->t[B->nt++];
        for (int j = 0; j < nsrc; j++) A.src[j] = src[t * nsrc + j];
        A.out = out[t];
        A.n = n[t];
        A.nt_store = nt_store();
        int nremote = __builtin_popcount(remote_mask[t] & ((1u << nsrc) - 1));
        *link += (double)n[t] * (double)es * nremote;
        *hbm += (double)n[t] * (double)es * (nsrc - nremote + 1);
    }
    *grid = B->nt ? ftar::plan_tree_batch(B, nsrc, es, d->max_blocks + 1) : 0;
    return 0;
}

} // namespace fdevi

extern "C" {

int fdev_tree_batch(ftar_dev *d, int dtype, int op, const void *const *src, int nsrc, const unsigned *remote_mask,
                    void *const *out, const size_t *n, int ntree, int tag)
{
    ftar::TreeBatch B;
    unsigned grid = 0;
    double link, hbm;
    int rc = build_batch(d, dtype, op, src, nsrc, remote_mask, out, n, ntree, tag, &B, &grid, &link, &hbm);
    if (rc || B.nt == 0) return rc;
    if (grid == 0) { // a tree beyond the workgroup budget: one (split) launch per tree
        for (int t = 0; t < ntree; t++) {
            int rc = fdev_tree(d, dtype, op, src + (size_t)t * nsrc, nsrc, remote_mask[t], out[t], n[t], tag);
            if (rc) return rc;
        }
        return 0;
    }
    d->ctr.link_bytes += link;
    d->ctr.hbm_bytes += hbm;
    note_launch(d, d->stream, grid, true, &B.sig);
    if (d->trace) {
        std::vector<TrRange> rd, wr;
        batch_ranges(B, nsrc, esize_of(dtype), rd, wr);
        tr_launch(d, d->stream, &B.sig, tr_rw(d, rd, wr), 0, "k");
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, d->stream);
    }
    hipError_t e = ftar::launch_tree_batch(dtype, op, nsrc, B, grid, d->stream);
    if (e != hipSuccess) return set_err(e, "tree_batch_kernel launch");
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, d->stream);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

int fdev_run(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    return run_on(d, d->stream, dtype, op, segs, nseg, tag);
}

} // extern "C"

extern "C" {

int fdev_run_bg(ftar_dev *d, int dtype, int op, const fdev_seg *segs, int nseg, int tag)
{
    int rc = ensure_bg(d);
    if (rc) return rc;
    hipEvent_t e = get_event(d);
    if (!e) return set_err(hipErrorOutOfMemory, "hipEventCreate");
    HIPCHK(hipEventRecord(e, d->stream));
    HIPCHK(hipStreamWaitEvent(d->bg, e, 0));
    d->event_pool.push_back(e);
    return run_on(d, d->bg, dtype, op, segs, nseg, tag);
}

int fdev_copy(ftar_dev *d, int bg, void *dst, const void *src, size_t bytes, int remote, int tag)
{
    if (tag < 0 || tag >= FDEV_NTAGS) return 13;
    if (bytes == 0) return 0;
    hipStream_t st = d->stream;
    if (bg) { // ordered after the main stream, like fdev_run_bg
        int rc = ensure_bg(d);
        if (rc) return rc;
        hipEvent_t e = get_event(d);
        if (!e) return set_err(hipErrorOutOfMemory, "hipEventCreate");
        HIPCHK(hipEventRecord(e, d->stream));
        HIPCHK(hipStreamWaitEvent(d->bg, e, 0));
        d->event_pool.push_back(e);
        st = d->bg;
    }
    if (remote) {
        d->ctr.link_bytes += (double)bytes;
        d->ctr.hbm_bytes += (double)bytes; // the local write
    } else {
        d->ctr.hbm_bytes += 2.0 * (double)bytes;
    }
    note_launch(d, st, ~0u, false, nullptr);
    if (d->trace) tr_launch(d, st, nullptr, tr_rw(d, {{src, bytes}}, {{dst, bytes}}), 0, "sdma");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (d->profiling) {
        e0 = get_event(d);
        e1 = get_event(d);
        if (e0) (void)hipEventRecord(e0, st);
    }
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    if (d->profiling && e0 && e1) {
        (void)hipEventRecord(e1, st);
        d->pending.push_back(Pending{e0, e1, tag});
    }
    return 0;
}

int fdev_order_after(ftar_dev *d, void *user_stream)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1); // nothing waits behind a closed gate
    // An idle caller stream has nothing our kernels must wait for (its kernels completed,
    // their stores released to this device).  A busy one is waited for on the host, never
    // by queuing a GPU-side dependency: an event recorded on the caller's stream is a
    // marker there, which the NEXT call's hipStreamQuery then finds pending (the runtime
    // reports completion of the caller's stream with a lag), so the wait was queued again
    // on every call -- and a cross-queue wait behind a marker on an otherwise idle queue
    // cost 30-50 us per call on one MI355X (tools/_exp_nullq.hip, profiles/r03/nullq/).
    // The call blocks until its own kernels are done anyway; waiting for the caller's
    // pending work first costs nothing extra.
    hipStream_t s = (hipStream_t)user_stream;
    hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) (void)hipGetLastError();
    d->user_host_waits++;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int fdev_user_host_waits(const ftar_dev *d) { return d->user_host_waits; }

} // extern "C"

namespace fdevi {

// Waits for everything enqueued on `st` by spinning on a fenced marker event.  Its
// system-scope sequentially consistent fence is what makes a step's results visible to
// the peers that pull them next -- the writeback puts this GPU's dirty L2 lines in HBM
// (peers read our HBM over xGMI, not our L2) -- and its invalidation drops this GPU's
// cached copies of peer memory, so the next step's pulls (issued after the barrier,
// with no peer reads in between) fetch the peers' new windows.  Without it the
// visibility of a kernel's stores to other GPUs would rest on the runtime's default
// packet fences.
int sync_stream(ftar_dev *d, hipStream_t st, int (*poll)(void *), void *arg)
{
    hipEvent_t fence = st == d->bg ? d->fence_bg : d->fence_main;
    if (d->tr_drop == 1) { // TEST-ONLY (FTAR_TRACE_DROP=release): the drain without its system fence
        hipEvent_t &nf = st == d->bg ? d->nofence_bg : d->nofence_main;
        if (!nf) HIPCHK(hipEventCreateWithFlags(&nf, hipEventDisableTiming | hipEventDisableSystemFence));
        fence = nf;
    }
    HIPCHK(hipEventRecord(fence, st));
    for (;;) {
        hipError_t e = hipEventQuery(fence);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return set_err(e, "hipEventQuery");
        if (poll) {
            int r = poll(arg);
            if (r) return r;
        }
    }
    tr(d, "D %s %c", d->tr_drop == 1 ? "nf" : "mk", st == d->bg ? 'b' : 'm');
    return 0;
}

// Waits for the signal of launch `tag` (its last workgroup's store into the pinned flag
// word), polling the failure detector; a device error surfaces through hipStreamQuery.
int wait_signal(ftar_dev *d, unsigned tag, int (*poll)(void *), void *arg)
{
    for (unsigned spins = 1;; spins++) {
        if ((int)(__atomic_load_n(d->sig_flag, __ATOMIC_ACQUIRE) - tag) >= 0) return 0;
        if (poll) {
            int r = poll(arg);
            if (r) return r;
        }
        if ((spins & 255) == 0) {
            hipError_t e = hipStreamQuery(d->stream);
            if (e == hipSuccess) { // the stream drained: the flag is there, or fall back
                if ((int)(__atomic_load_n(d->sig_flag, __ATOMIC_ACQUIRE) - tag) >= 0) return 0;
                return sync_stream(d, d->stream, poll, arg);
            }
            if (e != hipErrorNotReady) return set_err(e, "hipStreamQuery");
        }
    }
}

} // namespace fdevi

extern "C" {

int fdev_sync(ftar_dev *d, int (*poll)(void *), void *arg)
{
    int rc;
    if (d->gate_pending && d->big_pending) {
        // a mid-size launch waits on its closed gate: the fenced marker recorded just before
        // it covers (and released) everything queued earlier
        rc = spin(d->fence_pre, poll, arg);
        d->need_acquire = 0;
        d->pre_gate_any = 0;
        d->signalled = d->force_fence = 0;
        d->unsignalled = 1; // the gated launch, drained through a marker after its gate opens
        if (rc) return rc;
        tr(d, "D pre");
        rc = verify_gate(d, poll, arg);
        if (rc) return rc;
        return harvest(d);
    }
    if (d->gate_pending) {
        // a launch waits on its closed gate: drain what was queued before it (all of it
        // signalled, the gated launch checked; nothing is queued behind it, see note_launch),
        // never a marker behind the gate
        rc = d->pre_gate_any ? wait_signal(d, d->pre_gate_tag, poll, arg) : 0;
        if (!rc && d->pre_gate_any) tr(d, "D sig %u", d->pre_gate_tag);
        d->need_acquire = 1;
        d->pre_gate_any = 0;
        d->unsignalled = d->force_fence = 0;
        d->signalled = 1; // the gated launch, drained after its gate opens
        if (rc) return rc;
        // an earlier gated launch among them (RD: step s, opened; step s + 1 pending) has
        // completed too: check it now, before step s + 1 can read its result
        rc = verify_gate(d, poll, arg);
        if (rc) return rc;
        return harvest(d);
    }
    if (!d->unsignalled && !d->signalled && !d->force_fence) {
        rc = 0; // nothing queued since the last drain
    } else if (!d->unsignalled && d->signalled && !d->force_fence) {
        // only signalled launches: each workgroup released its stores at system scope before
        // the last one raised the flag, so the data is visible to the peers and the host
        rc = wait_signal(d, d->sig_tag, poll, arg);
        if (!rc) tr(d, "D sig %u", d->sig_tag);
        d->need_acquire = 1;
    } else {
        rc = sync_stream(d, d->stream, poll, arg);
        d->need_acquire = 0;
    }
    d->unsignalled = d->signalled = d->force_fence = 0;
    if (rc) return rc;
    rc = verify_gate(d, poll, arg); // the gated launch has completed: did its gate time out?
    if (rc) return rc;
    return harvest(d);
}

void fdev_fence_next_drain(ftar_dev *d) { d->force_fence = 1; }

int fdev_peer_wait(ftar_dev *d, void *flag, void *const *peer_flags, int npeers, uint64_t token,
                   int (*poll)(void *), void *arg)
{
    (void)poll;
    (void)arg;
    if (!d->sig_flag || !d->gate_dw || !flag || npeers < 1 || npeers > ftar::kMaxPeers) {
        snprintf(g_err, sizeof(g_err), "fdev_peer_wait: unavailable (%s) or bad arguments",
                 d->sig_flag ? "flag words" : "FTAR_FLAG_SYNC=0");
        return 13;
    }
    if (d->gate_pending) (void)fdev_gate_open(d, 1); // nothing waits behind a closed gate
    ftar::PeerWait W{};
    W.own = (unsigned long long *)flag;
    for (int i = 0; i < npeers; i++) W.peer[i] = (const unsigned long long *)peer_flags[i];
    W.npeers = npeers;
    W.token = (unsigned long long)token;
    d->pw_seq++;
    d->pw_vval = 2u * d->pw_seq;
    __atomic_store_n(d->sig_flag + 48, 0u, __ATOMIC_RELAXED); // verdict
    __atomic_store_n(d->sig_flag + 49, 0u, __ATOMIC_RELEASE); // abort word
    W.abort_word = d->sig_flag + 49;
    W.verdict_dev = d->gate_dw + 48;
    W.verdict_host = d->sig_flag + 48;
    W.vval = d->pw_vval;
    W.ticks = d->gate_ticks;
    // release: everything this rank queued so far is in HBM, device-wide, before its flag
    if (d->tr_drop == 1) { // TEST-ONLY (FTAR_TRACE_DROP=release): the flag without the release
        if (!d->nofence_main)
            HIPCHK(hipEventCreateWithFlags(&d->nofence_main, hipEventDisableTiming | hipEventDisableSystemFence));
        HIPCHK(hipEventRecord(d->nofence_main, d->stream));
    } else {
        HIPCHK(hipEventRecord(d->fence_main, d->stream));
    }
    if (d->trace) {
        std::string own, peers;
        tr_fmt(d, {{flag, 8}}, own);
        std::vector<TrRange> pr;
        for (int i = 0; i < npeers; i++) pr.push_back({peer_flags[i], 8});
        tr_fmt(d, pr, peers);
        if (d->tr_drop != 1) tr(d, "M pub"); // the fenced marker in front of the flag (a release, not a drain)
        tr(d, "F %llu w=%s", (unsigned long long)token, own.c_str());
        tr(d, "V %llu r=%s", (unsigned long long)token, peers.c_str());
    }
    hipError_t e = ftar::launch_peer_wait(W, d->stream);
    if (e != hipSuccess) return set_err(e, "peer_wait_kernel launch");
    d->unsignalled++; // drained through a fenced marker
    d->need_acquire = d->tr_drop == 1; // the marker invalidated the caches (unless it was dropped)
    d->pw_pending = 1;
    d->pw_armed = 0;
    return 0;
}

void fdev_peer_wait_abort(ftar_dev *d)
{
    if (d->sig_flag && d->pw_vval) __atomic_store_n(d->sig_flag + 49, d->pw_vval, __ATOMIC_RELEASE);
}

int fdev_peer_wait_verdict(ftar_dev *d)
{
    d->pw_pending = 0;
    if (!d->pw_armed) return 1;
    d->pw_armed = 0;
    if (__atomic_load_n(d->sig_flag + 48, __ATOMIC_ACQUIRE) == d->pw_vval) return 1;
    tr(d, "S %llu", d->pw_launch_n); // the launch behind the wait returned untouched
    return 0;
}

int fdev_busy(ftar_dev *d)
{
    hipError_t e = hipStreamQuery(d->stream);
    if (e == hipErrorNotReady) return 1;
    if (e != hipSuccess) (void)hipGetLastError();
    return 0;
}

int fdev_sync_bg(ftar_dev *d, int (*poll)(void *), void *arg)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1); // the background stream follows the main one
    if (!d->bg) return harvest(d); // never used: nothing queued
    int rc = sync_stream(d, d->bg, poll, arg);
    if (rc) return rc;
    return harvest(d);
}

} // extern "C"

namespace fdevi {

/* collect the timings of every event pair whose stop event has completed */
int harvest(ftar_dev *d)
{
    std::vector<Pending> still;
    for (auto &p : d->pending) {
        if (hipEventQuery(p.stop) != hipSuccess) {
            still.push_back(p);
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
            d->ctr.ms[p.tag] += ms;
            d->ctr.launches[p.tag]++;
        }
        d->event_pool.push_back(p.start);
        d->event_pool.push_back(p.stop);
    }
    d->pending.swap(still);
    return 0;
}

// The D2H copies ride on the background stream (idle in every call the pipeline runs
// in: it only carries a spare's redundancy copy, joined before each call returns), so a
// rank needs at most four streams -- null, main, background, H2D -- one hardware queue
// each (GPU_MAX_HW_QUEUES = 4); a fifth would share a queue and serialize the copies.
int ensure_pipe(ftar_dev *d)
{
    if (d->h2d) return 0;
    int rc = ensure_bg(d);
    if (rc) return rc;
    HIPCHK(hipStreamCreateWithFlags(&d->h2d, hipStreamNonBlocking));
    d->d2h = d->bg;
    // default (fenced) events: a landed chunk is visible to the peers that pull it
    for (int i = 0; i < FDEV_MAX_CHUNKS; i++) HIPCHK(hipEventCreateWithFlags(&d->h2d_done[i], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->fence_d2h, hipEventDisableTiming));
    return 0;
}

int spin(hipEvent_t e, int (*poll)(void *), void *arg)
{
    for (;;) {
        hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return 0;
        if (r != hipErrorNotReady) return set_err(r, "hipEventQuery");
        if (poll) {
            int rc = poll(arg);
            if (rc) return rc;
        }
    }
}

} // namespace fdevi

extern "C" {

int fdev_h2d_async(ftar_dev *d, void *dst, const void *src, size_t bytes, int slot)
{
    if (slot < 0 || slot >= FDEV_MAX_CHUNKS) return 13;
    int rc = ensure_pipe(d);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->h2d));
    HIPCHK(hipEventRecord(d->h2d_done[slot], d->h2d));
    return 0;
}

int fdev_wait_h2d(ftar_dev *d, int slot, int (*poll)(void *), void *arg)
{
    if (slot < 0 || slot >= FDEV_MAX_CHUNKS || !d->h2d) return 13;
    return spin(d->h2d_done[slot], poll, arg);
}

int fdev_d2h_async(ftar_dev *d, void *dst, const void *src, size_t bytes)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1);
    int rc = ensure_pipe(d);
    if (rc) return rc;
    hipEvent_t e = get_event(d);
    if (!e) return set_err(hipErrorOutOfMemory, "hipEventCreate");
    HIPCHK(hipEventRecord(e, d->stream));
    HIPCHK(hipStreamWaitEvent(d->d2h, e, 0));
    d->event_pool.push_back(e);
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->d2h));
    return 0;
}

int fdev_sync_d2h(ftar_dev *d, int (*poll)(void *), void *arg)
{
    if (d->gate_pending) (void)fdev_gate_open(d, 1);
    if (!d->d2h) return 0;
    HIPCHK(hipEventRecord(d->fence_d2h, d->d2h));
    return spin(d->fence_d2h, poll, arg);
}

int fdev_h2d(ftar_dev *d, void *dst, const void *src, size_t bytes)
{
    note_launch(d, d->stream, ~0u, false, nullptr);
    if (d->trace) tr_launch(d, d->stream, nullptr, tr_rw(d, {}, {{dst, bytes}}), 0, "h2d");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->stream));
    return fdev_sync(d, nullptr, nullptr);
}

int fdev_d2h(ftar_dev *d, void *dst, const void *src, size_t bytes)
{
    note_launch(d, d->stream, ~0u, false, nullptr);
    if (d->trace) tr_launch(d, d->stream, nullptr, tr_rw(d, {{src, bytes}}, {}), 0, "d2h");
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->stream));
    return fdev_sync(d, nullptr, nullptr);
}

} // extern "C"
