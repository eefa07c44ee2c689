"""DPDK wire frames for INT32 job slices (the second data type
of common.h:51-55).  The INT32 pre/post-processor only reorders bytes —
PreprocessSingle htonl's the block's words into the packet (ppp.cc:158-190),
PostprocessSingle ntohl's them out (ppp.cc:262-298) — and needs no extra
batch (NeedsExtraBatch is false, ppp.cc:65-67), so a slice has B frames and
frame p carries block p; the headers are BuildPacket's
(dpdk_worker_thread_utils.inc:67-135), the receive loop the worker's
(dpdk_worker_thread.cc:300-345: other job or pkt_id seen before -> discard).

CPU: the oracle's INT32 frames (orc_build_frames_i32 / orc_unpack_frames_i32)
against an independent numpy / Python restatement of the same rules.  GPU:
sml_pack_frames_int32 / sml_unpack_frames_int32 bit-exact against the
oracle — device and pinned frames, every packet size, misaligned slices,
shuffled streams with duplicates, other jobs' frames and out-of-range
pkt_ids, split rx calls — and the 16 M-element tx -> rx round trip.
"""
import struct

import numpy as np
import pytest

from oracle import oracle as O


def params(**kw):
    import switchml_amd as sw
    return sw.frame_params(**kw)


def int32_data(seed, n):
    return np.random.default_rng(seed).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)


def stream(frames, B, fb, seed, dup=0.1, wrong=0.05, bad=3, job=7):
    """A received stream of the slice's frames: shuffled, with late copies
    of some frames, frames of another job and pkt_ids >= B mixed in."""
    rng = np.random.default_rng(seed)
    fr = frames.reshape(B, fb)
    order = list(rng.permutation(B))
    order += list(rng.choice(B, int(dup * B) + 1))                      # duplicates, later
    out = [fr[i].copy() for i in order]
    for _ in range(int(wrong * B) + 1):                                  # another job's frame
        f = fr[rng.integers(B)].copy()
        f[43] = (job + 1) & 0xFF
        out.insert(int(rng.integers(len(out) + 1)), f)
    for _ in range(bad):                                                 # pkt_id past the slice
        f = fr[rng.integers(B)].copy()
        f[44:48] = np.frombuffer(struct.pack("<I", B + int(rng.integers(1, 1000))), dtype=np.uint8)
        out.insert(int(rng.integers(len(out) + 1)), f)
    return np.concatenate(out)


# ---------------------------------------------------------------- CPU --

@pytest.mark.parametrize("P,n", [(256, 3000), (64, 1), (1024, 5000)])
def test_oracle_int32_frames_fields(P, n):
    fp = params(job_id=0x1207, pool_index_start=64, pool_index_shift=10, max_outstanding_pkts=8)
    x = int32_data(P + n, n)
    f = O.build_frames_i32(x, fp, P=P)
    fl = O.build_frames(np.zeros(n, dtype=np.float32), fp, P=P, batch_max=8)    # FLOAT32 frames: same headers
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    assert f.size == B * fb
    for p in range(B):
        fr = f[p * fb:(p + 1) * fb].tobytes()
        assert fr[:44] == fl[:44].tobytes()                         # Eth / IPv4 / UDP / job_type_size / job id
        assert struct.unpack("<I", fr[44:48])[0] == p               # pkt_id, host order, no extra batch
        assert struct.unpack(">H", fr[48:50])[0] == O.pool_index(p, 64, 10, 8)
        assert fr[50:52] == b"\0\0"                                 # no exponent for INT32
        valid = min(P, n - p * P)
        words = np.frombuffer(fr[52:], dtype=">i4")                 # network order on the wire
        assert np.array_equal(words[:valid].astype(np.int32), x[p * P:p * P + valid])
        assert not words[valid:].any()


def python_rx(stream_bytes, fb, n, P, job, seen, out):
    """The receive loop restated in Python (dpdk_worker_thread.cc:300-345 with
    the INT32 PostprocessSingle)."""
    B = O.num_blocks(n, P)
    acc = dis = 0
    for i in range(len(stream_bytes) // fb):
        fr = stream_bytes[i * fb:(i + 1) * fb]
        pid = struct.unpack("<I", fr[44:48].tobytes())[0]
        if pid >= B or seen[pid] or fr[43] != (job & 0xFF):
            dis += 1
            continue
        seen[pid] = 1
        acc += 1
        valid = min(P, n - pid * P)
        out[pid * P:pid * P + valid] = np.frombuffer(fr[52:52 + 4 * valid].tobytes(), dtype=">i4")
    return acc, dis


@pytest.mark.parametrize("P,n", [(256, 20_011), (64, 777), (1024, 3 * 1024)])
def test_oracle_int32_rx_loop(P, n):
    fp = params(job_id=7, max_outstanding_pkts=16)
    x = int32_data(3 * n, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    s = stream(O.build_frames_i32(x, fp, P=P), B, fb, seed=n)
    half = (len(s) // fb // 2) * fb
    rx = O.RxStateI32(n, P)
    seen = np.zeros(B, dtype=np.uint8)
    ref = np.zeros(n, dtype=np.int32)
    acc = dis = 0
    for part in (s[:half], s[half:]):                                    # two rx calls of one slice
        O.unpack_frames_i32(part, part.size // fb, fb, rx, job_id=7)
        a, d = python_rx(part, fb, n, P, 7, seen, ref)
        acc, dis = acc + a, dis + d
    assert np.array_equal(rx.out, ref) and np.array_equal(rx.out, x)
    assert rx.counts == [acc, dis] and acc == B


def test_rx_state_words():
    """sml_rx_state_words: the rx state a receive call needs (host-only)."""
    import switchml_amd as sw
    L = sw.lib()
    for n, P, bm in [(0, 256, 64), (1, 64, 64), (20_011, 256, 64), (3 * 1024, 1024, 2), (10 ** 9 + 7, 128, 512)]:
        B = O.num_blocks(n, P)
        assert L.sml_rx_state_words(n, P, bm, 1) == 2 * B + 6        # + the fix-up's dirty list
        assert L.sml_rx_state_words(n, P, bm, 0) == max(1, B + min(B, bm))
    assert L.sml_rx_state_words(1000, 100, 64, 0) == 0          # unsupported packet size
    assert sw.RxSliceInt32(20_011, 256, device="cpu").state.numel() == 2 * O.num_blocks(20_011, 256) + 6


# ---------------------------------------------------------------- GPU --

@pytest.mark.gpu
@pytest.mark.parametrize("P", [64, 128, 256, 512, 1024])
@pytest.mark.parametrize("n", [1, 300, 50_003])
@pytest.mark.parametrize("where", ["device", "pinned"])
def test_int32_frames_match_oracle(cuda, P, n, where):
    import torch
    import switchml_amd as sw
    fp = params(job_id=9, pool_index_start=16, pool_index_shift=3, max_outstanding_pkts=32)
    x = int32_data(n + P, n)
    ref = O.build_frames_i32(x, fp, P=P)
    B = O.num_blocks(n, P)
    stride = 52 + 4 * P + 12          # mbuf-like padding between frames; padding bytes untouched
    if where == "device":
        frames = torch.full((B * stride,), 0xAB, dtype=torch.uint8, device=cuda)
    else:
        frames = torch.full((B * stride,), 0xAB, dtype=torch.uint8).pin_memory()
    sw.pack_frames_int32(torch.from_numpy(x).to(cuda), fp, P, frames=frames, stride=stride)
    torch.cuda.synchronize()
    got = frames.cpu().numpy().reshape(B, stride)
    bad = np.argwhere(got[:, :52 + 4 * P] != ref.reshape(B, 52 + 4 * P))
    assert bad.size == 0, (bad[:8].tolist(), got[bad[0][0], :64].tolist() if bad.size else None,
                           ref.reshape(B, 52 + 4 * P)[bad[0][0], :64].tolist() if bad.size else None)
    assert np.all(got[:, 52 + 4 * P:] == 0xAB)


@pytest.mark.gpu
@pytest.mark.parametrize("nt", [False, True])
def test_int32_frames_misaligned_slice_and_store_policy(cuda, nt):
    """A FIFO slice starting 4 bytes past a 16-B boundary; the non-temporal
    payload-store policy (threshold 0) gives the same bytes."""
    import torch
    import switchml_amd as sw
    P, n = 256, 40_001
    fp = params(job_id=300, max_outstanding_pkts=64)
    full = int32_data(5, n + 3)
    xd = torch.from_numpy(full).to(cuda)[3:]
    assert xd.data_ptr() % 16 != 0
    orig = sw.set_payload_nt_threshold(0 if nt else 2 ** 64 - 1)
    try:
        got = sw.pack_frames_int32(xd, fp, P)
        torch.cuda.synchronize()
    finally:
        sw.set_payload_nt_threshold(orig)
    assert np.array_equal(got.cpu().numpy(), O.build_frames_i32(full[3:], fp, P=P))


@pytest.mark.gpu
@pytest.mark.parametrize("P,n", [(256, 100_003), (64, 4_099), (1024, 30_001), (128, 1), (512, 2 * 512)])
@pytest.mark.parametrize("where", ["device", "pinned"])
def test_int32_rx_streams_match_oracle(cuda, P, n, where):
    """Shuffled received frames with late duplicates, other jobs' frames and
    pkt_ids past the slice, in two rx calls of one slice: output words and
    {accepted, discarded} bit-exact with the oracle loop."""
    import torch
    import switchml_amd as sw
    fp = params(job_id=7, max_outstanding_pkts=16)
    x = int32_data(7 * n + P, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    s = stream(O.build_frames_i32(x, fp, P=P), B, fb, seed=n + P)
    nfr = s.size // fb
    cut = nfr // 2
    ref = O.RxStateI32(n, P)
    rx = sw.RxSliceInt32(n, P, device=cuda)
    rx.reset()
    for lo, hi in ((0, cut), (cut, nfr)):
        part = s[lo * fb:hi * fb]
        O.unpack_frames_i32(part, hi - lo, fb, ref, job_id=7)
        t = torch.from_numpy(part.copy())
        t = t.to(cuda) if where == "device" else t.pin_memory()
        sw.unpack_frames_int32(t, hi - lo, rx, job_id=7)
    torch.cuda.synchronize()
    assert np.array_equal(rx.out.cpu().numpy(), ref.out)
    assert np.array_equal(ref.out, x)
    assert rx.counts.cpu().tolist() == ref.counts


@pytest.mark.gpu
def test_int32_frames_round_trip_16M(cuda):
    """16 M INT32 words (64 MiB): tx frames -> rx in one call, the identity;
    every word back, every frame accepted."""
    import torch
    import switchml_amd as sw
    n, P = 16 * 1024 * 1024 + 5, 256
    fp = params(job_id=3)
    g = torch.Generator(device=cuda)
    g.manual_seed(11)
    x = torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), dtype=torch.int32, device=cuda, generator=g)
    frames = sw.pack_frames_int32(x, fp, P)
    B = sw.num_blocks(n, P)
    rx = sw.RxSliceInt32(n, P, device=cuda)
    rx.reset()
    sw.unpack_frames_int32(frames, B, rx, job_id=3)
    torch.cuda.synchronize()
    assert torch.equal(rx.out, x)
    assert rx.counts.cpu().tolist() == [B, 0]


def altered_copies_stream(frames, B, fb, seed, pairs, max_gap=4096):
    """The slice's frames in order, plus for `pairs` pkt_ids a copy whose
    payload differs (words XOR 0x5A5A5A5A), inserted a random 1..max_gap
    frames before or after the original: the first copy in stream order must
    win whichever copy the GPU claims first."""
    rng = np.random.default_rng(seed)
    fr = [f.copy() for f in frames.reshape(B, fb)]
    pos = {p: float(p) for p in range(B)}
    extra = []
    for p in rng.choice(B, min(pairs, B), replace=False):
        alt = fr[p].copy()
        alt[52:] ^= 0x5A
        gap = int(rng.integers(1, max_gap + 1)) * (1 if rng.random() < 0.5 else -1)
        extra.append((pos[p] + gap + 0.5 * np.sign(gap), alt))
    items = [(pos[p], fr[p]) for p in range(B)] + extra
    items.sort(key=lambda it: it[0])
    return np.concatenate([f for _, f in items])


@pytest.mark.gpu
@pytest.mark.parametrize("P,n,pairs", [(64, 4 * 1024 * 1024, 20_000), (256, 8 * 1024 * 1024 + 3, 8_000),
                                       (1024, 2 * 1024 * 1024, 1_000)])
def test_int32_rx_first_copy_wins_over_racing_copies(cuda, P, n, pairs):
    """Copies of a pkt_id with DIFFERENT payloads, one before or after the
    original at random distances, in one rx call: the one-pass kernel claims
    in whatever order the waves run; the output must be the first copy's
    words (the reference loop's rule) and the counts exact."""
    import torch
    import switchml_amd as sw
    fp = params(job_id=5)
    x = int32_data(P + 17, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    s = altered_copies_stream(O.build_frames_i32(x, fp, P=P), B, fb, seed=P, pairs=pairs)
    nfr = s.size // fb
    seen = np.zeros(B, dtype=np.uint8)
    ref = np.zeros(n, dtype=np.int32)
    acc, dis = python_rx(s, fb, n, P, 5, seen, ref)
    rx = sw.RxSliceInt32(n, P, device=cuda)
    rx.reset()
    sw.unpack_frames_int32(torch.from_numpy(s).to(cuda), nfr, rx, job_id=5)
    torch.cuda.synchronize()
    got = rx.out.cpu().numpy()
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, (bad.size, bad[:8].tolist())
    assert rx.counts.cpu().tolist() == [acc, dis] and acc == B and dis == pairs
    st = rx.state.cpu().numpy()
    assert st[B] == 1 and st[B + 3] == 0 and st[B + 5] == 0   # call sequence advanced, call 1's slot clear
    assert not (st[:B] & 1).any()                              # no dirty pkt_id left
    print(f"P={P}: {rx.conflicts} of {pairs} copies claimed ahead of an earlier copy")


def lead_stream(x, fp, P, K, pairs_iters, other_job):
    """A stream shaped for ONE workgroup of 4 waves (grid limit 1: wave w
    takes tiles w, w + 4, ... of F = 1024 / P frames, P >= 256 here): for K
    iterations wave 0's tiles hold distinct valid frames (claim + store) and
    waves 1-3's tiles another job's frames (no claim), so wave 1 runs ahead;
    then for `pairs_iters` iterations wave 0's tile holds the first copies of
    F pkt_ids and wave 1's tile later, altered copies of the same pkt_ids —
    which wave 1 reaches first.  Returns the stream bytes."""
    F = 1024 // P
    fb = 52 + 4 * P
    B = O.num_blocks(x.size, P)
    fr = O.build_frames_i32(x, fp, P=P).reshape(B, fb)
    other = fr[0].copy()
    other[43] = other_job
    tiles = []
    pid = 0
    for _ in range(K):
        tiles.append([fr[pid + j] for j in range(F)])
        pid += F
        tiles += [[other] * F] * 3
    for _ in range(pairs_iters):
        first = [fr[pid + j] for j in range(F)]
        alt = [f.copy() for f in first]
        for a in alt:
            a[52:] ^= 0x5A
        tiles += [first, alt, [other] * F, [other] * F]
        pid += F
    assert pid <= B
    return np.concatenate([f for t in tiles for f in t])


@pytest.mark.gpu
@pytest.mark.parametrize("P", [256, 1024])
def test_int32_rx_racing_copies_smoke(cuda, P):
    """A SMOKE TEST of real scheduling, not the pin of the fix-up (VERDICT r5
    #5): a stream laid out so that later copies of pkt_ids (different
    payloads) tend to reach the claim atomic before the earlier copies (their
    wave runs ahead).  Asserted: the output is the first copies' words and the
    counts are exact, whatever the scheduling did.  NOT asserted: that any
    later copy actually claimed first — the hardware decides the interleaving
    of waves, so the number that did (printed) can be 0 on a given run
    (r05z: 0 of 256; other runs: all of them).  No launch order makes it
    deterministic: a frame's tag is its position in the call, and one wave
    walks its tiles in that order, so only a cross-wave race can put a later
    copy first.  The fix-up itself is pinned, deterministically, by
    test_int32_rx_fixup_rewrites_displaced_claims (pre-seeded later claims)."""
    import torch
    import switchml_amd as sw
    K, pairs_iters = 3000, 64
    F = 1024 // P
    n = (K + pairs_iters) * F * P
    fp = params(job_id=5)
    x = int32_data(P, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    s = lead_stream(x, fp, P, K, pairs_iters, other_job=6)
    nfr = s.size // fb
    seen = np.zeros(B, dtype=np.uint8)
    ref = np.zeros(n, dtype=np.int32)
    acc, dis = python_rx(s, fb, n, P, 5, seen, ref)
    assert np.array_equal(ref, x)                               # every first copy is the original
    old_lim, old_xcd = sw.set_grid_limit(1), sw.set_xcd_chunk(0)
    try:
        rx = sw.RxSliceInt32(n, P, device=cuda)
        rx.reset()
        sw.unpack_frames_int32(torch.from_numpy(s).to(cuda), nfr, rx, job_id=5)
        torch.cuda.synchronize()
    finally:
        sw.set_grid_limit(old_lim)
        sw.set_xcd_chunk(old_xcd)
    got = rx.out.cpu().numpy()
    bad = np.flatnonzero(got != ref)
    assert bad.size == 0, (bad.size, bad[:8].tolist())
    assert rx.counts.cpu().tolist() == [acc, dis]
    # a scheduling fact, not a correctness one: reported, never asserted
    print(f"P={P}: {rx.conflicts} of {pairs_iters * F} later copies claimed first (smoke: any number passes)")


def claim_tag(call, f):
    """k_rx_int32's claim tag (sml_frames.hip rx_int32_tag) as a signed int64."""
    t = ((0xFFFFFFFF - call) << 32) | ((0x7FFFFFFF - f) << 1)
    return int(np.array(t, dtype=np.uint64).view(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("overflow", [False, True])
@pytest.mark.parametrize("P", [64, 256, 1024])
def test_int32_rx_fixup_rewrites_displaced_claims(cuda, P, overflow):
    """The fix-up path, white box: before the call, some pkt_ids hold the
    claim tag of a LATER frame of this call (as when a later copy wins the
    race to the atomic) and their output words hold that copy's garbage.  The
    real (earlier) frames must displace those claims, mark them dirty, and
    the fix-up must leave the earlier frames' words, clean state words, the
    conflict count in the slice total, and the call sequence advanced.  The
    fix-up visits the call's dirty list (state[B + 4 ...]);
    overflow=True plants a full list first, so every append is dropped and
    the fix-up takes its fallback, the scan of all B state words."""
    import torch
    import switchml_amd as sw
    n = 40_000 + 7
    fp = params(job_id=4)
    x = int32_data(P + 3, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    frames = O.build_frames_i32(x, fp, P=P)
    rng = np.random.default_rng(P)
    stolen = np.sort(rng.choice(B, max(1, B // 5), replace=False))
    rx = sw.RxSliceInt32(n, P, device=cuda)
    rx.reset()
    st = rx.state.cpu().numpy()
    for k in stolen:                                    # frame k's later twin (index B + k) claimed k first
        st[k] = claim_tag(0, B + int(k))
    if overflow:
        st[B + 4] = B                                   # call 0's list is full: the fix-up must scan
    rx.state.copy_(torch.from_numpy(st))
    rx.out.fill_(-1)
    sw.unpack_frames_int32(torch.from_numpy(frames).to(cuda), B, rx, job_id=4)
    torch.cuda.synchronize()
    assert np.array_equal(rx.out.cpu().numpy(), x)
    st = rx.state.cpu().numpy()
    assert not (st[:B] & 1).any()
    # sequence, slice total, call 0's conflict count and list length (left:
    # the next fix-up clears them), call 1's (cleared)
    assert [int(v) for v in st[B:B + 6]] == [1, len(stolen), len(stolen), 0,
                                             B + len(stolen) if overflow else len(stolen), 0]
    if not overflow:                                    # each displaced pkt_id listed once, in some order
        assert sorted(int(v) for v in st[B + 6:B + 6 + len(stolen)]) == [int(k) for k in stolen]
    assert rx.conflicts == len(stolen)
    # displaced claims count as the discards (their twins were counted accepted)
    assert rx.counts.cpu().tolist() == [B - len(stolen), len(stolen)]
    # a second call: every pkt_id is now held by call 0, so all copies are discarded
    rx.out.fill_(0)
    sw.unpack_frames_int32(torch.from_numpy(frames).to(cuda), B, rx, job_id=4)
    torch.cuda.synchronize()
    assert not rx.out.cpu().numpy().any()
    assert rx.counts.cpu().tolist() == [B - len(stolen), B + len(stolen)]
    assert int(rx.state[B].item()) == 2


@pytest.mark.gpu
def test_int32_rx_many_calls_keep_earlier_winners(cuda):
    """Seven rx calls of one slice, each a shuffled part of a stream with
    altered copies: a pkt_id accepted by an earlier call discards every later
    copy (no retirement pass: the call sequence orders the tags)."""
    import torch
    import switchml_amd as sw
    P, n = 256, 300_001
    fp = params(job_id=9)
    x = int32_data(99, n)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    s = altered_copies_stream(O.build_frames_i32(x, fp, P=P), B, fb, seed=3, pairs=600, max_gap=B)
    nfr = s.size // fb
    cuts = np.sort(np.random.default_rng(4).choice(np.arange(1, nfr), 6, replace=False))
    bounds = [0, *cuts.tolist(), nfr]
    seen = np.zeros(B, dtype=np.uint8)
    ref = np.zeros(n, dtype=np.int32)
    acc = dis = 0
    rx = sw.RxSliceInt32(n, P, device=cuda)
    rx.reset()
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        part = s[lo * fb:hi * fb]
        a, d = python_rx(part, fb, n, P, 9, seen, ref)
        acc, dis = acc + a, dis + d
        sw.unpack_frames_int32(torch.from_numpy(part.copy()).to(cuda), hi - lo, rx, job_id=9)
    torch.cuda.synchronize()
    assert np.array_equal(rx.out.cpu().numpy(), ref)
    assert rx.counts.cpu().tolist() == [acc, dis]
    assert int(rx.state[B].item()) == len(bounds) - 1


@pytest.mark.gpu
def test_int32_rx_scattered_pids_over_1GiB_output(cuda):
    """An INT32 slice whose output passes 1 GiB, received with every wave's
    frames interleaving pkt_ids from the two halves (half a GiB apart and
    more): the non-temporal output stores must reach every address (a buffer
    store spanning +-1 GiB around a wave's first lane would drop them)."""
    import torch
    import switchml_amd as sw
    P = 256
    n = (1 << 28) + 1000
    fp = params(job_id=2)
    g = torch.Generator(device=cuda)
    g.manual_seed(5)
    x = torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), dtype=torch.int32, device=cuda, generator=g)
    B = sw.num_blocks(n, P)
    fb = sw.frame_bytes(P)
    frames = sw.pack_frames_int32(x, fp, P).view(B, fb)
    h = B // 2
    order = torch.stack([torch.arange(h, device=cuda), torch.arange(h, 2 * h, device=cuda)], 1).flatten()
    order = torch.cat([order, torch.arange(2 * h, B, device=cuda)])
    shuffled = frames.index_select(0, order).flatten()
    del frames
    rx = sw.RxSliceInt32(n, P, device=cuda)
    rx.reset()
    sw.unpack_frames_int32(shuffled, B, rx, job_id=2)
    torch.cuda.synchronize()
    assert rx.counts.cpu().tolist() == [B, 0]
    assert torch.equal(rx.out, x)


@pytest.mark.gpu
def test_int32_rx_random_streams(cuda):
    """Randomized INT32 receive streams (Hypothesis, derandomized): any P,
    slice length, 1-5 rx calls, copies with altered payloads before or after
    the original, other jobs' frames, pkt_ids past the slice, frames missing
    — output words and counts equal the sequential first-copy-wins loop after
    every call."""
    pytest.importorskip("hypothesis")
    import torch
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    import switchml_amd as sw

    @settings(max_examples=60, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
    @given(n=st.integers(0, 30_000), P=st.sampled_from([64, 128, 256, 512, 1024]), job=st.integers(0, 255),
           pairs=st.integers(0, 40), wrong=st.integers(0, 4), bad=st.integers(0, 3), drop=st.integers(0, 5),
           calls=st.integers(1, 5), seed=st.integers(0, 2 ** 31))
    def check(n, P, job, pairs, wrong, bad, drop, calls, seed):
        rng = np.random.default_rng(seed)
        fp = params(job_id=job)
        fb = 52 + 4 * P
        B = O.num_blocks(n, P)
        x = int32_data(seed, n)
        if B:
            frames = O.build_frames_i32(x, fp, P=P)
            s = altered_copies_stream(frames, B, fb, seed, pairs=min(pairs, B), max_gap=max(1, B))
            rows = list(s.reshape(-1, fb))
            for _ in range(min(drop, len(rows) - 1)):                  # frames that never arrive
                rows.pop(int(rng.integers(len(rows))))
            other = frames[:fb].copy()
        else:
            rows = []
            other = np.zeros(fb, dtype=np.uint8)
            other[43] = job
        for _ in range(wrong):
            f = other.copy()
            f[43] = (job + 1) & 0xFF
            rows.insert(int(rng.integers(len(rows) + 1)), f)
        for _ in range(bad):
            f = other.copy()
            f[43] = job & 0xFF
            f[44:48] = np.frombuffer(struct.pack("<I", B + int(rng.integers(0, 5))), dtype=np.uint8)
            rows.insert(int(rng.integers(len(rows) + 1)), f)
        if not rows:
            return
        s = np.concatenate(rows)
        nfr = len(rows)
        cuts = sorted(set(int(c) for c in rng.integers(1, nfr, calls - 1))) if nfr > 1 and calls > 1 else []
        bounds = [0, *cuts, nfr]
        seen = np.zeros(max(B, 1), dtype=np.uint8)
        ref = np.zeros(n, dtype=np.int32)
        acc = dis = 0
        rx = sw.RxSliceInt32(n, P, device=cuda)
        rx.reset()
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            part = s[lo * fb:hi * fb]
            a, d = python_rx(part, fb, n, P, job, seen, ref)
            acc, dis = acc + a, dis + d
            sw.unpack_frames_int32(torch.from_numpy(part.copy()).to(cuda), hi - lo, rx, job_id=job)
            torch.cuda.synchronize()
            assert np.array_equal(rx.out.cpu().numpy(), ref), (n, P, lo, hi)
            assert rx.counts.cpu().tolist() == [acc, dis], (n, P, lo, hi)
        assert int(rx.state[O.num_blocks(n, P)].item()) == len(bounds) - 1          # call sequence
    check()


@pytest.mark.gpu
def test_int32_frames_random_parameters(cuda):
    """Randomized INT32 frame builds (Hypothesis, derandomized): any P,
    length, job id, pool start / shift / max outstanding, padding,
    misalignment, device or pinned frames — every byte equal to the oracle."""
    pytest.importorskip("hypothesis")
    import torch
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    import switchml_amd as sw

    @settings(max_examples=50, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
    @given(n=st.integers(1, 20_000), P=st.sampled_from([64, 128, 256, 512, 1024]),
           job=st.integers(0, 2 ** 16 - 1), start=st.integers(0, 2 ** 15 - 1), shift=st.integers(0, 4000),
           mop=st.integers(1, 512), pad=st.sampled_from([0, 4, 12, 60]), off=st.integers(0, 3),
           pinned=st.booleans(), seed=st.integers(0, 2 ** 31))
    def check(n, P, job, start, shift, mop, pad, off, pinned, seed):
        fp = params(job_id=job, pool_index_start=start, pool_index_shift=shift, max_outstanding_pkts=mop)
        full = int32_data(seed, n + off)
        ref = O.build_frames_i32(full[off:], fp, P=P)
        B = O.num_blocks(n, P)
        stride = 52 + 4 * P + pad
        frames = torch.full((B * stride,), 0xAB, dtype=torch.uint8)
        frames = frames.pin_memory() if pinned else frames.to(cuda)
        sw.pack_frames_int32(torch.from_numpy(full).to(cuda)[off:], fp, P, frames=frames, stride=stride)
        torch.cuda.synchronize()
        got = frames.cpu().numpy().reshape(B, stride)
        assert np.array_equal(got[:, :52 + 4 * P], ref.reshape(B, 52 + 4 * P)), (n, P, off)
        assert np.all(got[:, 52 + 4 * P:] == 0xAB)
    check()
