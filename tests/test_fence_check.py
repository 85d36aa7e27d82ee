"""tests/fence_check.py (the cross-device fence-discipline checker of the FTAR_TRACE logs) on
synthetic two-rank logs: a mesh-like call that follows the rules passes; the same call with
one release dropped (an unfenced drain) fails the release rule; a read of a peer window
that was cached by a read before the barrier, with no fenced marker or acquire since, fails
the acquire rule.  The GPU test (tests/test_gpu_fences.py) runs the checker on the
library's own logs."""
import os

import fence_check as FC


def L(n, w="-", r="-", sig=0, acq=0, fence=0, gate=0, sw="-", stag=0, s="m", eng="k"):
    rel = 1 if sig else 0
    return f"L {n} s={s} sig={sig} rel={rel} acq={acq} fence={fence} gate={gate} eng={eng} r={r} w={w} sw={sw} stag={stag}"


def _call(me, peer, k0, drain_tree="D mk m", ag_acq=0, second_drain="D mk m", tag0=1):
    """One two-launch mesh call of rank `me`: stage IN (signalled), barrier, tree over the
    peer's IN into my W block, drain, barrier, allgather pull of the peer's W block, drain,
    barrier.  Rank r owns W bytes [64 r, 64 r + 64)."""
    mine, theirs = 64 * me, 64 * peer
    return [L(1 + 3 * (k0 // 3), w=f"{me}:IN:0:128,", sig=tag0), f"D sig {tag0}", f"A {k0}", f"P {k0}",
            L(2 + 3 * (k0 // 3), r=f"{me}:IN:{mine}:64,{peer}:IN:{mine}:64,", w=f"{me}:W:{mine}:64,"), drain_tree,
            f"A {k0 + 1}", f"P {k0 + 1}",
            L(3 + 3 * (k0 // 3), r=f"{peer}:W:{theirs}:64,", acq=ag_acq), second_drain, f"A {k0 + 2}", f"P {k0 + 2}"]


def _write(tmp, logs):
    for r, lines in logs.items():
        with open(os.path.join(tmp, f"t.{r}"), "w") as f:
            f.write("# ftar trace: device 0, flag_sync 1, drop 0\n" + "\n".join(lines) + "\n")
    return os.path.join(tmp, "t")


def test_clean_mesh_calls_pass(tmp_path):
    pre = _write(str(tmp_path), {0: _call(0, 1, 1) + _call(0, 1, 4, tag0=2), 1: _call(1, 0, 1) + _call(1, 0, 4, tag0=2)})
    rep = FC.check_prefix(pre)
    assert rep.ok, (rep.release, rep.acquire)
    assert rep.reads_checked >= 4


def test_dropped_release_is_caught(tmp_path):
    pre = _write(str(tmp_path), {0: _call(0, 1, 1), 1: _call(1, 0, 1, drain_tree="D nf m")})
    rep = FC.check_prefix(pre)
    assert rep.release and "rank 0" in rep.release[0] and "rank 1's launch" in rep.release[0], rep.release
    assert not rep.acquire


def test_missing_acquire_is_caught(tmp_path):
    # call 2's allgather read of the peer's block follows only flag drains: the lines call 1's
    # allgather cached may be stale, and the launch does not invalidate
    def call2(me, peer):
        c = _call(me, peer, 4, drain_tree="D sig 3", tag0=2)
        c[4] = c[4].replace("sig=0 rel=0", "sig=3 rel=1")  # the tree signalled: a flag drain
        return c

    c1 = {r: _call(r, 1 - r, 1, second_drain="D sig 1") for r in (0, 1)}
    logs = {r: c1[r] + call2(r, 1 - r) for r in (0, 1)}
    rep = FC.check_prefix(_write(str(tmp_path), logs))
    assert rep.acquire and "without an acquire" in rep.acquire[0], (rep.acquire, rep.release)
    # the same with the allgather invalidating itself (signal_acquire) passes
    logs = {r: c1[r] + [x.replace("acq=0", "acq=1") if x.startswith("L 6") else x for x in call2(r, 1 - r)]
            for r in (0, 1)}
    rep = FC.check_prefix(_write(str(tmp_path), logs))
    assert not rep.acquire, rep.acquire


def test_gated_launch_runs_at_its_gate(tmp_path):
    """A gated launch's body runs when its gate opens (G go), after the barrier; a skipped
    one never runs; the staging phase before the gate is released by its own flag."""
    def rank(me, peer, skip=False):  # the one-shot form: stages IN, then reads the peer's IN into rbuf
        return [L(1, r=f"{peer}:IN:0:128,", sig=2, acq=1, gate=1, sw=f"{me}:IN:0:128,", stag=1),
                "D sig 1", "A 1", "P 1", f"G 1 {'skip' if skip else 'go'}", "D sig 2", "A 2", "P 2"]
    rep = FC.check_prefix(_write(str(tmp_path), {0: rank(0, 1), 1: rank(1, 0)}))
    assert rep.ok and rep.reads_checked == 2, (rep.release, rep.acquire)
    # the staging's release not waited for before the barrier: caught
    bad = rank(1, 0)
    bad[1] = "D sig 0"
    rep = FC.check_prefix(_write(str(tmp_path), {0: rank(0, 1), 1: bad}))
    assert rep.release, rep


def test_dead_rank_reads(tmp_path):
    """A rank that died before the reader's barrier: what it wrote before its last arrival
    must have been released by then (a recovery reads it: the replay of its step-0 input),
    and what it wrote after (its in-flight step) must never be read."""
    dead = ["A 1", "P 1", L(1, w="1:IN:0:64,", sig=1), "D sig 1", "A 2", "P 2", L(2, w="1:W:0:64,")]
    live = ["A 1", "P 1", "A 2", "P 2", "A 3", "P 3", L(5, r="1:IN:0:64,")]
    rep = FC.check_prefix(_write(str(tmp_path), {0: live, 1: dead}))
    assert rep.ok and rep.dead_reads == 1, (rep.release, rep.dead_reads)
    live[-1] = L(5, r="1:W:0:64,")  # the dead rank's unreleased in-flight step read
    rep = FC.check_prefix(_write(str(tmp_path), {0: live, 1: dead}))
    assert rep.release and "after its last arrival" in rep.release[0], rep.release


def _devwait_call(me, peer, k0, pub="M pub", wait=True, tok=None):
    """The mesh with the allgather ordered on the device (fdev_peer_wait): stage, barrier k0,
    tree into my W block, fenced marker + flag F, wait V for the peer's flag, allgather of the
    peer's W block behind a fenced marker, drain, barrier k0 + 1."""
    mine, theirs = 64 * me, 64 * peer
    tok = k0 if tok is None else tok
    lines = [L(1, w=f"{me}:IN:0:128,", sig=1), "D sig 1", f"A {k0}", f"P {k0}",
             L(2, r=f"{me}:IN:{mine}:64,{peer}:IN:{mine}:64,", w=f"{me}:W:{mine}:64,")]
    if pub:
        lines.append(pub)
    lines += [f"F {k0} w={me}:W:4096:8,"]
    if wait:
        lines.append(f"V {tok} r={peer}:W:4096:8,")
    lines += [L(3, r=f"{peer}:W:{theirs}:64,", fence=1), "D mk m", f"A {k0 + 1}", f"P {k0 + 1}"]
    return lines


def test_device_wait_orders_the_allgather(tmp_path):
    """The allgather reads the peer's block written in the same round: fine behind a wait for
    the peer's flag that a fenced marker released the tree in front of."""
    rep = FC.check_prefix(_write(str(tmp_path), {0: _devwait_call(0, 1, 1), 1: _devwait_call(1, 0, 1)}))
    assert rep.ok, (rep.release, rep.acquire)
    assert rep.reads_checked >= 4


def test_device_wait_without_release_is_caught(tmp_path):
    """FTAR_TRACE_DROP=release on the flag's marker: the tree was not released before the flag."""
    rep = FC.check_prefix(_write(str(tmp_path), {0: _devwait_call(0, 1, 1), 1: _devwait_call(1, 0, 1, pub=None)}))
    assert rep.release and "no fenced marker released it before flag" in rep.release[0], rep.release


def test_same_round_read_without_wait_is_a_race(tmp_path):
    """The allgather queued without the wait (no V): it reads what the peer writes in the same
    round -- a race the barrier rule alone never sees."""
    rep = FC.check_prefix(_write(str(tmp_path), {0: _devwait_call(0, 1, 1, wait=False), 1: _devwait_call(1, 0, 1)}))
    assert rep.release and "in the same round, with no wait" in rep.release[0], rep.release
    # a wait for a token the peer never published
    rep = FC.check_prefix(_write(str(tmp_path), {0: _devwait_call(0, 1, 1, tok=7), 1: _devwait_call(1, 0, 1)}))
    assert rep.release and "never published" in rep.release[0], rep.release


def test_skipped_launch_reads_nothing(tmp_path):
    """A launch behind a wait that was given up (S n) returned untouched: nothing it would
    have read is checked."""
    r0 = _devwait_call(0, 1, 1, wait=False)
    r0.insert(r0.index("D mk m") + 1, "S 3")
    rep = FC.check_prefix(_write(str(tmp_path), {0: r0, 1: _devwait_call(1, 0, 1)}))
    assert rep.ok, rep.release
