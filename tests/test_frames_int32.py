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
