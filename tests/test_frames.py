"""DPDK wire frames: the fused quantize-into-frames kernel
against the oracle's restatement of BuildPacket + PreprocessSingle
(client_lib/src/backends/dpdk/dpdk_worker_thread_utils.inc:42-135,
ppp.cc:69-156).  Byte-exact over every frame's data_len bytes.

DPDK itself is an un-vendored submodule (DPDK 20.x, make-based build; commit
not recorded) and is not in the image, so its two helpers on this path are
restated from their published algorithms: rte_ipv4_phdr_cksum = rte_raw_cksum
(ones-complement 16-bit sum, folded, not inverted) of the 12-byte pseudo
header; header field layouts = rte_ether_hdr / rte_ipv4_hdr / rte_udp_hdr.
"""
import socket
import struct

import numpy as np
import pytest

from oracle import oracle as O


def params(**kw):
    import switchml_amd as sw
    return sw.frame_params(**kw)


# ---------------------------------------------------------------- CPU --

def test_oracle_frame_fields():
    P, n, W = 256, 3000, 2
    fp = params(job_id=0x1234, pool_index_start=64, pool_index_shift=10, max_outstanding_pkts=8,
                src_ip="10.0.0.1", dst_ip="10.0.0.253", src_port=4000, dst_port=48879)
    x = O.splitmix_normal(1, n)
    f = O.build_frames(x, fp, P=P, num_workers=W, batch_max=8)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    b = min(B, 8)
    assert f.size == (B + b) * fb
    exps = O.exponents(x, P)
    q = O.quantize(x, P, W)
    for p in range(B + b):
        fr = f[p * fb:(p + 1) * fb].tobytes()
        assert fr[0:6] == bytes([2, 0, 0, 0, 0, 1]) and fr[6:12] == bytes([2, 0, 0, 0, 0, 2])
        assert fr[12:14] == b"\x08\x00"
        ver, tos, tot = struct.unpack(">BBH", fr[14:18])
        assert (ver, tot) == (0x45, fb - 14)
        assert fr[22] == 128 and fr[23] == 17
        assert fr[26:30] == socket.inet_aton("10.0.0.1") and fr[30:34] == socket.inet_aton("10.0.0.253")
        sport, dport, ulen = struct.unpack(">HHH", fr[34:40])
        assert (sport, dport, ulen) == (4000, 48879, fb - 34)
        # pseudo-header sum, stored as rte_raw_cksum leaves it (memory-order words)
        psd = fr[26:34] + bytes([0, 17]) + struct.pack(">H", fb - 34)
        s = sum(struct.unpack("<6H", psd))
        s = (s & 0xFFFF) + (s >> 16)
        s = (s & 0xFFFF) + (s >> 16)
        assert struct.unpack("<H", fr[40:42])[0] == s
        assert fr[42] == (1 << 4) + 3 and fr[43] == 0x34
        assert struct.unpack("<I", fr[44:48])[0] == p
        assert struct.unpack(">H", fr[48:50])[0] == O.pool_index(p, 64, 10, 8)
        assert fr[50] == (int(exps[p]) & 0xFF if p < B else 0) and fr[51] == 0
        payload = np.frombuffer(fr[52:], dtype=np.uint32)
        if p >= b:
            k = p - b
            valid = min(P, n - k * P)
            assert np.array_equal(payload[:valid], q[k * P:k * P + valid])
        else:
            assert not payload.any()


def test_pool_index_alternates_shadow_pools():
    """PktId2PoolIndex: ids cycle over 2*mop slots, the upper half with the MSB set."""
    mop, start = 4, 100
    got = [O.pool_index(p, start, 0, mop) for p in range(10)]
    assert got == [100, 101, 102, 103, 0x8064, 0x8065, 0x8066, 0x8067, 100, 101]
    assert O.pool_index(0, start, 5, mop) == 0x8065


# ---------------------------------------------------------------- GPU --

@pytest.mark.gpu
@pytest.mark.parametrize("P", [64, 256, 1024])
@pytest.mark.parametrize("n", [1, 300, 50_003])
@pytest.mark.parametrize("where", ["device", "pinned"])
@pytest.mark.parametrize("nt", [False, True])
def test_frames_match_oracle(cuda, P, n, where, nt):
    """nt: the non-temporal payload-store policy (device frame sets from the
    threshold on; threshold 0 here) — the same bytes."""
    import torch
    import switchml_amd as sw
    orig = sw.set_payload_nt_threshold(0 if nt else 2 ** 64 - 1)
    try:
        _frames_match_oracle(cuda, P, n, where)
    finally:
        sw.set_payload_nt_threshold(orig)


def _frames_match_oracle(cuda, P, n, where):
    import torch
    import switchml_amd as sw
    W, bm = 3, 16
    fp = params(job_id=7, pool_index_start=16, pool_index_shift=3, max_outstanding_pkts=bm)
    x = O.splitmix_normal(n + P, n)
    ref = O.build_frames(x, fp, P=P, num_workers=W, batch_max=bm)
    B = O.num_blocks(n, P)
    b = min(B, bm)
    stride = 52 + 4 * P + 12   # mbuf-like padding between frames; padding bytes untouched
    if where == "device":
        frames = torch.full(((B + b) * stride,), 0xAB, dtype=torch.uint8, device=cuda)
    else:
        frames = torch.full(((B + b) * stride,), 0xAB, dtype=torch.uint8).pin_memory()
    sw.quantize_pack_frames(torch.from_numpy(x).to(cuda), fp, P, W, batch_max=bm, frames=frames, stride=stride)
    torch.cuda.synchronize()
    got = frames.cpu().numpy().reshape(B + b, stride)
    exp = ref.reshape(B + b, 52 + 4 * P)
    assert np.array_equal(got[:, :52 + 4 * P], exp)
    assert np.all(got[:, 52 + 4 * P:] == 0xAB)


@pytest.mark.gpu
def test_frames_global_exponents_and_misaligned_slice(cuda):
    import torch
    import switchml_amd as sw
    P, n, W, bm = 256, 40_001, 2, 64
    fp = params(job_id=300, max_outstanding_pkts=bm)
    xfull = O.splitmix_normal(5, n + 3)
    x = xfull[3:]
    B = O.num_blocks(n, P)
    ge = np.clip(O.exponents(x, P).astype(np.int32) + 1, -128, 127).astype(np.int8)
    ref = O.build_frames(x, fp, P=P, num_workers=W, batch_max=bm, global_exps=ge)
    xd = torch.from_numpy(xfull).to(cuda)[3:]
    assert xd.data_ptr() % 16 != 0
    got = sw.quantize_pack_frames(xd, fp, P, W, batch_max=bm, global_exps=torch.from_numpy(ge).to(cuda))
    assert np.array_equal(got.cpu().numpy(), ref)


@pytest.mark.gpu
def test_frames_random_parameters(cuda):
    """Randomized frame builds (Hypothesis, derandomized): any P, slice
    length, W, batch, job id, pool start / shift / max outstanding, frame
    padding, misalignment of the slice, global exponents or not, device or
    pinned frames — every byte equal to the oracle's BuildPacket +
    PreprocessSingle, padding untouched."""
    pytest.importorskip("hypothesis")
    import torch
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st
    import switchml_amd as sw

    @settings(max_examples=60, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))
    @given(n=st.integers(1, 20_000), P=st.sampled_from([64, 128, 256, 512, 1024]), W=st.integers(1, 9),
           bm=st.integers(1, 300), job=st.integers(0, 2 ** 16 - 1), start=st.integers(0, 2 ** 15 - 1),
           shift=st.integers(0, 4000), mop=st.integers(1, 512), pad=st.sampled_from([0, 4, 12, 60]),
           off=st.integers(0, 3), glob=st.booleans(), pinned=st.booleans(), seed=st.integers(0, 2 ** 31))
    def check(n, P, W, bm, job, start, shift, mop, pad, off, glob, pinned, seed):
        fp = params(job_id=job, pool_index_start=start, pool_index_shift=shift, max_outstanding_pkts=mop)
        xfull = O.splitmix_normal(seed, n + off) * np.float32(2.0 ** ((seed % 40) - 20))
        x = xfull[off:]
        B = O.num_blocks(n, P)
        b = min(B, bm)
        ge = None
        if glob:
            ge = np.clip(O.exponents(x, P).astype(np.int32) + (seed % 3), -128, 127).astype(np.int8)
        ref = O.build_frames(x, fp, P=P, num_workers=W, batch_max=bm, global_exps=ge)
        stride = 52 + 4 * P + pad
        frames = torch.full(((B + b) * stride,), 0xAB, dtype=torch.uint8)
        frames = frames.pin_memory() if pinned else frames.to(cuda)
        xd = torch.from_numpy(xfull).to(cuda)[off:]
        sw.quantize_pack_frames(xd, fp, P, W, batch_max=bm, frames=frames, stride=stride,
                                global_exps=None if ge is None else torch.from_numpy(ge).to(cuda))
        torch.cuda.synchronize()
        got = frames.cpu().numpy().reshape(B + b, stride)
        assert np.array_equal(got[:, :52 + 4 * P], ref.reshape(B + b, 52 + 4 * P)), (n, P, W, bm, off)
        assert np.all(got[:, 52 + 4 * P:] == 0xAB)
    check()


# ------------------------------------------------------- RDMA (F4) -----

def rdma_imm_reference(exps, batch_max):
    """rdma_worker_thread.cc:341-356: imm = msg_id & 0xFFFF, then
    PreprocessSingle writes the exponent into byte 2 (messages m < B)."""
    B = exps.size
    total = B + min(B, batch_max)
    imm = np.zeros(total, dtype=np.uint32)
    for m in range(total):
        word = bytearray(struct.pack("<I", m & 0xFFFF))
        if m < B:
            word[2] = int(exps[m]) & 0xFF
        imm[m] = struct.unpack("<I", bytes(word))[0]
    return imm


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000, 1024 * 70_000 + 5])
def test_rdma_messages(cuda, n):
    """1024-element RDMA messages: payload = the P = 1024 planes, exponent in
    the immediate's byte 2; msg ids past 65535 wrap in the low 16 bits."""
    import torch
    import switchml_amd as sw
    P, W, bm = 1024, 2, 32
    x = O.splitmix_normal(11, n)
    payload, exps = sw.quantize_pack(torch.from_numpy(x).to(cuda), P, W)
    assert np.array_equal(payload.cpu().numpy().view(np.uint32), O.quantize(x, P, W))
    imm = sw.rdma_imm(exps, bm).cpu().numpy().view(np.uint32)
    assert np.array_equal(imm, rdma_imm_reference(O.exponents(x, P), bm))
    # an INT32 slice of the same size: B messages, the immediate is the msg id alone
    B = exps.numel()
    imm_i = sw.rdma_imm(None, num_blocks_int32=B, device=cuda).cpu().numpy().view(np.uint32)
    assert np.array_equal(imm_i, (np.arange(B) & 0xFFFF).astype(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["pinned", "device"])
def test_per_packet_bursts_into_mbufs_equal_bulk_frames(cuda, where):
    """A DPDK worker that keeps the per-packet PPP calls (BuildPacket by the
    host, then PreprocessSingle into the mbuf: payload at offset 52, extra
    info at offset 50 — dpdk_worker_thread_utils.inc:132-134) and runs them in
    bursts, interleaved with PostprocessSingle of the returned packets as the
    receive loop does (dpdk_worker_thread.cc:300-345), leaves exactly the
    frames the fused frames kernel writes in bulk: the two entry points agree
    byte for byte on the wire."""
    import torch
    import switchml_amd as sw
    P, n, bm = 256, 50_003, 64
    fp = params(job_id=3, max_outstanding_pkts=bm)
    x = O.splitmix_normal(77, n)
    want = O.build_frames(x, fp, P=P, batch_max=bm)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    b = min(B, bm)
    total = B + b
    # BuildPacket's part: the headers; the PPP's part (exponent byte, payload) blank
    pre = want.reshape(total, fb).copy()
    pre[:, 50] = 0
    pre[:, 52:] = 0
    frames = torch.from_numpy(pre.reshape(-1).copy())
    frames = frames.to(cuda) if where == "device" else frames.pin_memory()
    base = frames.data_ptr()
    xd = torch.from_numpy(x).to(cuda)
    out = torch.full((n,), float("nan"), device=cuda)
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    stream = torch.cuda.current_stream(cuda)

    def burst(ids, pre_call):
        if not ids:
            return
        bt = sw.packet_burst(xd, out, P, 1, b, recv, ids, [base + p * fb + 52 for p in ids],
                             [base + p * fb + 50 for p in ids])
        (sw.preprocess_burst if pre_call else sw.postprocess_burst)(bt, stream)

    burst(list(range(b)), True)
    for p0 in range(0, total, b):
        ids = list(range(p0, min(p0 + b, total)))
        burst(ids, False)                                            # the switch returned them unchanged (W = 1)
        burst([q + b for q in ids if q + b < total], True)           # ReusePacket -> the next packet
    torch.cuda.synchronize()
    got = frames.cpu().numpy()
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad.size, [(int(i) // fb, int(i) % fb) for i in bad[:8]])
    _, _, ref_out, _ = O.dummy_packet_stream(x, P=P, batch_max=bm, num_workers=1)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref_out.view(np.uint32))


@pytest.mark.gpu
def test_per_packet_int32_bursts_into_mbufs_equal_bulk_frames(cuda):
    """The same for an INT32 slice (no extra batch, no exponent): per-packet
    bursts into mbuf-layout frames == sml_pack_frames_int32, and the receive
    side's bursts give the words back."""
    import torch
    import switchml_amd as sw
    P, n = 256, 30_011
    fp = params(job_id=6)
    xi = np.random.default_rng(8).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
    want = O.build_frames_i32(xi, fp, P=P)
    fb = 52 + 4 * P
    B = O.num_blocks(n, P)
    pre = want.reshape(B, fb).copy()
    pre[:, 52:] = 0
    frames = torch.from_numpy(pre.reshape(-1).copy()).pin_memory()
    base = frames.data_ptr()
    xd = torch.from_numpy(xi).to(cuda)
    out = torch.zeros(n, dtype=torch.int32, device=cuda)
    for p0 in range(0, B, sw.MAX_BURST):
        ids = list(range(p0, min(p0 + sw.MAX_BURST, B)))
        bt = sw.packet_burst(xd, out, P, 1, 0, None, ids, [base + p * fb + 52 for p in ids],
                             [base + p * fb + 50 for p in ids])
        sw.preprocess_burst(bt)
        sw.postprocess_burst(bt)
    torch.cuda.synchronize()
    assert np.array_equal(frames.numpy(), want)
    assert np.array_equal(out.cpu().numpy(), xi)
