"""Per-packet calls in bursts (sml_preprocess_burst / sml_postprocess_burst,
csrc/sml_packets.hip): the reference's PreprocessSingle / PostprocessSingle
(ppp.cc:69-192, 194-299) for a DPDK-style rx burst and the tx burst it
refills (dpdk_worker_thread.cc:276-345, dpdk_worker_thread_utils.inc:134,177).

The driver here is the reference's dummy packet loop (dummy_worker_thread.cc:
86-177) with its ring of b packet slots — in pinned host memory (a NIC's
buffer pool) and in HBM — run burst by burst; packets inside a burst in
shuffled order.  Every packet as sent (exponent byte for p < B, the n real
payload words for p >= b) is captured after its burst and compared with the
oracle's packet-loop capture (orc_dummy_packet_stream), the output with the
oracle's output, bit for bit; the stale tail words of a partial last block
must be left as they were.  Plus INT32 slices and the argument checks."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O


def sw():
    import switchml_amd as s
    s.lib()
    return s


def run_bursts(x, P, W, b_max, ring_place, cuda, rng, burst_cap=64):
    """The dummy packet loop, burst by burst, through the C-ABI; returns
    (captured packet exps, captured packet payloads, output, b)."""
    import torch
    s = sw()
    n = x.size
    B = O.num_blocks(n, P)
    b = min(B, b_max)
    total = B + b
    xd = torch.from_numpy(x).to(cuda)
    out = torch.full((n,), float("nan"), device=cuda)
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    SENT = 0x5A5A5A5A                        # the slots' bytes before any packet was built
    if ring_place == "device":
        ring = torch.full((b * P,), SENT, dtype=torch.int64, device=cuda).to(torch.int32)
        extra = torch.zeros(b * 2, dtype=torch.uint8, device=cuda)
    else:
        ring = torch.full((b * P,), SENT, dtype=torch.int64).to(torch.int32).pin_memory()
        extra = torch.zeros(b * 2, dtype=torch.uint8).pin_memory()
    rbase, ebase = ring.data_ptr(), extra.data_ptr()
    cap_e = np.zeros(total, dtype=np.int8)
    cap_p = np.zeros((total, P), dtype=np.uint32)
    stream = torch.cuda.current_stream(cuda)

    def bursts(ids, pre):
        ids = list(ids)
        rng.shuffle(ids)                       # a burst's packets in any order
        for i0 in range(0, len(ids), burst_cap):
            part = ids[i0:i0 + burst_cap]
            slots = [q % b for q in part]
            bt = s.packet_burst(xd, out, P, W, b, recv, part, [rbase + sl * P * 4 for sl in slots],
                                [ebase + sl * 2 for sl in slots])
            (s.preprocess_burst if pre else s.postprocess_burst)(bt, stream)
        torch.cuda.synchronize()

    def snapshot():
        return ring.cpu().numpy().view(np.uint32).reshape(b, P).copy()

    def capture(ids, before):
        rh = snapshot()
        eh = extra.cpu().numpy()
        for q in ids:
            sl = q % b
            cap_e[q] = eh[sl * 2].astype(np.int8) if q < B else 0
            if q >= b:
                m = min(P, n - (q - b) * P)
                cap_p[q, :m] = rh[sl, :m]
                # a partial block's tail keeps the slot's stale words (ppp.cc:102-109)
                assert np.array_equal(rh[sl, m:], before[sl, m:]), "stale tail overwritten"

    prev = snapshot()
    bursts(range(b), True)
    capture(range(b), prev)
    for p0 in range(0, total, b):
        w = min(b, total - p0)
        torch.cuda.synchronize()
        rh = ring.view(torch.int32)
        # ProcessPacket x W (dummy_backend.cc:72-84) on the window's slots
        if W != 1:
            s.loopback_aggregate(rh[: w * P], W)
        torch.cuda.synchronize()
        bursts(range(p0, p0 + w), False)
        nxt = [q + b for q in range(p0, p0 + w) if q + b < total]
        prev = snapshot()
        bursts(nxt, True)
        capture(nxt, prev)
    return cap_e, cap_p, out.cpu().numpy(), b


@pytest.mark.gpu
@pytest.mark.parametrize("P,W,n,b_max,ring,cap", [
    (256, 1, 40_000, 64, "device", 64),
    (256, 3, 100_003, 64, "pinned", 64),
    (64, 2, 12_345, 50, "pinned", 17),
    (1024, 8, 70_001, 16, "device", 64),
    (128, 1, 777, 64, "device", 5),        # B < b_max: b = B
    (512, 3, 513, 64, "pinned", 64),
])
def test_burst_loop_matches_oracle_packet_stream(cuda, P, W, n, b_max, ring, cap):
    rng = np.random.default_rng(P + W + n)
    x = O.splitmix_normal(n % 97, n) * np.float32(2.0 ** (W - 2))
    if n > 1000:
        x[100:140] = 0.0                             # an all-zero-ish stretch, special values
        x[5] = np.float32(2.5)
        x[6] = np.float32(-2.5)
    pe, pp, ref_out, b = O.dummy_packet_stream(x, P=P, batch_max=b_max, num_workers=W)
    ce, cp, out, b2 = run_bursts(x, P, W, b_max, ring, cuda, rng, cap)
    assert b == b2
    assert np.array_equal(ce, pe)
    assert np.array_equal(cp, pp.view(np.uint32))
    assert np.array_equal(out.view(np.uint32), ref_out.view(np.uint32))


@pytest.mark.gpu
def test_burst_int32_and_argument_checks(cuda):
    import torch
    s = sw()
    P, n = 256, 5_000
    xi = np.random.default_rng(3).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
    xd = torch.from_numpy(xi).to(cuda)
    outd = torch.zeros_like(xd)
    B = O.num_blocks(n, P)
    pk = torch.zeros(B * P, dtype=torch.int32, device=cuda)
    ids = list(range(B))
    bt = s.packet_burst(xd, outd, P, 1, 0, None, ids, [pk.data_ptr() + q * P * 4 for q in ids], [0] * B)
    s.preprocess_burst(bt)
    s.postprocess_burst(bt)
    torch.cuda.synchronize()
    assert np.array_equal(pk.cpu().numpy().view(np.uint32)[:n], O.bswap32(xi))
    assert np.array_equal(outd.cpu().numpy(), xi)
    # a float burst holding q and q + b, a duplicate id, an id past B + b, > MAX_BURST packets
    x = torch.randn(10_000, device=cuda)
    o = torch.empty_like(x)
    Bf = O.num_blocks(10_000, P)
    recv = torch.zeros(Bf, dtype=torch.int8, device=cuda)
    ring = torch.zeros(64 * P, dtype=torch.int32, device=cuda)
    ex = torch.zeros(128, dtype=torch.uint8, device=cuda)
    for bad in ([3, 3 + 8], [4, 4], [Bf + 8]):
        bt = s.packet_burst(x, o, P, 1, 8, recv, bad, [ring.data_ptr()] * len(bad), [ex.data_ptr()] * len(bad))
        with pytest.raises(s.SwitchMLError):
            s.preprocess_burst(bt)
    bt = s.packet_burst(x, o, P, 1, 8, recv, [0], [ring.data_ptr()], [ex.data_ptr()])
    bt.count = 65
    with pytest.raises(s.SwitchMLError):
        s.postprocess_burst(bt)


@pytest.mark.gpu
@pytest.mark.parametrize("W,Q,ring", [(1, 16, "pinned"), (3, 16, "device"), (2, 5, "pinned")])
def test_rdma_message_loop_with_immediate_words(cuda, W, Q, ring):
    """The RDMA worker's loop (rdma_worker_thread.cc:205-262, 330-356) through
    the burst calls: 1024-element messages in Q queue-pair slots; message m
    posts from slot m % Q with imm_data = m & 0xFFFF and PreprocessSingle's
    extra info at imm byte 2 (:345-351); on receipt the short id is checked
    and PostprocessSingle reads the exponent from the received imm byte 2
    (:223-244), then slot m % Q is refilled with message m + Q.  The kernels
    must write ONLY imm byte 2 (the message id in bytes 0-1 survives, byte 3
    stays 0), and every message and the output must equal the oracle's packet
    loop with b = Q."""
    import torch
    s = sw()
    P, n = 1024, 70_001
    x = O.splitmix_normal(W + Q, n) * np.float32(3.0)
    pe, pp, ref_out, b = O.dummy_packet_stream(x, P=P, batch_max=Q, num_workers=W)
    B = O.num_blocks(n, P)
    assert b == min(B, Q)
    total = B + b
    xd = torch.from_numpy(x).to(cuda)
    out = torch.full((n,), float("nan"), device=cuda)
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    msgs = torch.zeros(b * P, dtype=torch.int32)
    imm = torch.zeros(b, dtype=torch.int32).pin_memory()          # one imm word per queue pair
    msgs = msgs.to(cuda) if ring == "device" else msgs.pin_memory()
    stream = torch.cuda.current_stream(cuda)
    cap_e = np.zeros(total, dtype=np.int8)
    cap_p = np.zeros((total, P), dtype=np.uint32)

    def burst(ids, pre):
        bt = s.packet_burst(xd, out, P, W, b, recv, ids, [msgs.data_ptr() + (m % b) * P * 4 for m in ids],
                            [imm.data_ptr() + 4 * (m % b) + 2 for m in ids])
        (s.preprocess_burst if pre else s.postprocess_burst)(bt, stream)
        torch.cuda.synchronize()

    def post_sends(ids):                                          # PostSendWr for each message
        iv = imm.numpy().view(np.uint32)
        for m in ids:
            iv[m % b] = m & 0xFFFF
        burst(ids, True)
        iv = imm.numpy().view(np.uint32)
        mh = msgs.cpu().numpy().view(np.uint32).reshape(b, P)
        for m in ids:
            assert iv[m % b] & 0xFFFF == m & 0xFFFF and iv[m % b] >> 24 == 0, (m, hex(int(iv[m % b])))
            cap_e[m] = np.int8(np.uint8((iv[m % b] >> 16) & 0xFF)) if m < B else 0
            if m >= b:
                k = m - b
                cap_p[m, :min(P, n - k * P)] = mh[m % b, :min(P, n - k * P)]

    post_sends(list(range(b)))
    for p0 in range(0, total, b):
        ids = list(range(p0, min(p0 + b, total)))
        if W != 1:                                                 # the switch: x W on the payload words
            s.loopback_aggregate(msgs.view(torch.int32)[: len(ids) * P], W)
            torch.cuda.synchronize()
        iv = imm.numpy().view(np.uint32)
        assert all(iv[m % b] & 0xFFFF == m & 0xFFFF for m in ids)   # the expected short message ids
        burst(ids, False)                                          # PostprocessSingle(imm byte 2)
        post_sends([m + b for m in ids if m + b < total])
    assert np.array_equal(cap_e, pe)
    assert np.array_equal(cap_p, pp.view(np.uint32))
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref_out.view(np.uint32))


def run_exchange(x, P, W, b_max, ring_place, cuda, rng, burst_cap=64, proc_in_kernel=True):
    """The same packet loop with one sml_exchange_burst per pass (post of p
    and pre of p + b into the slot, in one launch — DPDK's receive loop +
    ReusePacket); ProcessPacket x W inside it (FLAG_PROCESS_PACKET) or as a
    separate K5 launch first."""
    import torch
    s = sw()
    n = x.size
    B = O.num_blocks(n, P)
    b = min(B, b_max)
    total = B + b
    xd = torch.from_numpy(x).to(cuda)
    out = torch.full((n,), float("nan"), device=cuda)
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    SENT = 0x5A5A5A5A
    if ring_place == "device":
        ring = torch.full((b * P,), SENT, dtype=torch.int64, device=cuda).to(torch.int32)
        extra = torch.zeros(b * 2, dtype=torch.uint8, device=cuda)
    else:
        ring = torch.full((b * P,), SENT, dtype=torch.int64).to(torch.int32).pin_memory()
        extra = torch.zeros(b * 2, dtype=torch.uint8).pin_memory()
    rbase, ebase = ring.data_ptr(), extra.data_ptr()
    cap_e = np.zeros(total, dtype=np.int8)
    cap_p = np.zeros((total, P), dtype=np.uint32)
    stream = torch.cuda.current_stream(cuda)

    def snapshot():
        return ring.cpu().numpy().view(np.uint32).reshape(b, P).copy()

    def processed(words):
        return O.bswap32((O.bswap32(words).astype(np.uint64) * W % (1 << 32)).astype(np.uint32))

    def capture(ids, before):
        rh = snapshot()
        eh = extra.cpu().numpy()
        for q in ids:
            sl = q % b
            cap_e[q] = eh[sl * 2].astype(np.int8) if q < B else 0
            if q >= b:
                m = min(P, n - (q - b) * P)
                cap_p[q, :m] = rh[sl, :m]
                assert np.array_equal(rh[sl, m:], before[sl, m:]), "tail words not as ProcessPacket left them"

    ids0 = list(range(b))
    prev = snapshot()
    for i0 in range(0, b, burst_cap):
        part = ids0[i0:i0 + burst_cap]
        s.preprocess_burst(s.packet_burst(xd, out, P, W, b, recv, part, [rbase + q * P * 4 for q in part],
                                          [ebase + q * 2 for q in part]), stream)
    torch.cuda.synchronize()
    capture(ids0, prev)
    for p0 in range(0, total, b):
        w = min(b, total - p0)
        if W != 1 and not proc_in_kernel:
            s.loopback_aggregate(ring.view(torch.int32)[: w * P], W)
        torch.cuda.synchronize()
        before = snapshot()
        if proc_in_kernel:
            before = processed(before)
        ids = list(range(p0, p0 + w))
        rng.shuffle(ids)
        for i0 in range(0, w, burst_cap):
            part = ids[i0:i0 + burst_cap]
            slots = [q % b for q in part]
            bt = s.packet_burst(xd, out, P, W, b, recv, part, [rbase + sl * P * 4 for sl in slots],
                                [ebase + sl * 2 for sl in slots],
                                flags=s.FLAG_PROCESS_PACKET if proc_in_kernel else 0)
            s.exchange_burst(bt, stream)
        torch.cuda.synchronize()
        capture([q + b for q in range(p0, p0 + w) if q + b < total], before)
    return cap_e, cap_p, out.cpu().numpy(), b


@pytest.mark.gpu
@pytest.mark.parametrize("P,W,n,b_max,ring,cap,proc", [
    (256, 1, 40_000, 64, "device", 64, True),
    (256, 3, 100_003, 64, "device", 64, True),
    (256, 3, 100_003, 64, "pinned", 64, False),
    (64, 2, 12_345, 50, "pinned", 17, True),
    (1024, 8, 70_001, 16, "device", 64, False),
    (1024, 5, 70_001, 16, "pinned", 7, True),
    (128, 1, 777, 64, "device", 5, True),          # B < b_max: b = B
    (512, 3, 513, 64, "pinned", 64, False),
])
def test_exchange_loop_matches_oracle_packet_stream(cuda, P, W, n, b_max, ring, cap, proc):
    rng = np.random.default_rng(P * 7 + W + n)
    x = O.splitmix_normal(n % 89, n) * np.float32(2.0 ** (W - 2))
    if n > 1000:
        x[100:140] = 0.0
        x[5] = np.float32(2.5)
        x[6] = np.float32(-2.5)
    pe, pp, ref_out, b = O.dummy_packet_stream(x, P=P, batch_max=b_max, num_workers=W)
    ce, cp, out, b2 = run_exchange(x, P, W, b_max, ring, cuda, rng, cap, proc)
    assert b == b2
    assert np.array_equal(ce, pe)
    assert np.array_equal(cp, pp.view(np.uint32))
    assert np.array_equal(out.view(np.uint32), ref_out.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("ring", ["device", "pinned"])
def test_exchange_int32_window_and_argument_checks(cuda, ring):
    import torch
    s = sw()
    P, n, b = 256, 20_000, 8
    xi = np.random.default_rng(5).integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
    xd = torch.from_numpy(xi).to(cuda)
    outd = torch.zeros_like(xd)
    B = O.num_blocks(n, P)
    slots = torch.zeros(b * P, dtype=torch.int32, device=cuda if ring == "device" else "cpu")
    if ring == "pinned":
        slots = slots.pin_memory()
    base = slots.data_ptr()
    # INT32: packet q carries block q; the first b packets, then every received
    # packet q is post'ed and its buffer refilled with block q + b
    first = list(range(b))
    s.preprocess_burst(s.packet_burst(xd, outd, P, 1, 0, None, first, [base + q * P * 4 for q in first], [0] * b))
    for p0 in range(0, B, b):
        ids = list(range(p0, min(p0 + b, B)))
        s.exchange_burst(s.packet_burst(xd, outd, P, 1, b, None, ids, [base + (q % b) * P * 4 for q in ids],
                                        [0] * len(ids)))
    torch.cuda.synchronize()
    assert np.array_equal(outd.cpu().numpy(), xi)
    # refused: window 0, q and q + b in one burst, an id past B + b (FLOAT32)
    x = torch.randn(10_000, device=cuda)
    o = torch.empty_like(x)
    Bf = O.num_blocks(10_000, P)
    recv = torch.zeros(Bf, dtype=torch.int8, device=cuda)
    rg = torch.zeros(64 * P, dtype=torch.int32, device=cuda)
    ex = torch.zeros(128, dtype=torch.uint8, device=cuda)
    for bw, bad in ((0, [1]), (8, [3, 11]), (8, [Bf + 8])):
        bt = s.packet_burst(x, o, P, 1, bw, recv, bad, [rg.data_ptr()] * len(bad), [ex.data_ptr()] * len(bad))
        with pytest.raises(s.SwitchMLError):
            s.exchange_burst(bt)


@pytest.mark.gpu
@pytest.mark.parametrize("P,W,n,b_max,ring,seed,server", [
    (256, 2, 60_001, 64, "device", 1, False),
    (256, 3, 33_333, 32, "pinned", 2, False),
    (1024, 8, 50_000, 16, "device", 3, False),
    (64, 1, 9_999, 48, "pinned", 4, False),
    (256, 3, 33_333, 32, "pinned", 5, True),
    (1024, 5, 50_000, 16, "pinned", 6, True),
    (128, 2, 20_001, 64, "device", 7, True),
])
def test_exchange_random_delivery_like_dummy_backend(cuda, P, W, n, b_max, ring, seed, server):
    """DummyBackend::ReceiveBurst delivers a RANDOM subset of the pending
    packets in random order (dummy_backend.cc:99-118: k = rand() % (pending +
    1), each a random pending index), ProcessPacket (x W) on receipt; the
    worker then post-processes each received packet and refills its slot with
    packet p + b (dummy_worker_thread.cc:125-170).  The same loop here, every
    receive burst one sml_exchange_burst with FLAG_PROCESS_PACKET: each packet
    as sent and the output equal the oracle's in-order packet stream bit for
    bit (slots are independent, so the delivery order cannot change a byte).
    Before every receive, up to three outstanding packets are re-built into
    spare buffers, as the DPDK timeout path re-sends them, and must equal the
    packets in flight byte for byte.  `server`: every burst goes through the
    persistent burst server (sml_burst_server_submit) instead of a launch."""
    import torch
    s = sw()
    rng = np.random.default_rng(seed)
    x = O.splitmix_normal(seed + 11, n) * np.float32(2.0 ** (seed - 2))
    pe, pp, ref_out, b = O.dummy_packet_stream(x, P=P, batch_max=b_max, num_workers=W)
    B = O.num_blocks(n, P)
    total = B + b
    xd = torch.from_numpy(x).to(cuda)
    out = torch.full((n,), float("nan"), device=cuda)
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    if ring == "device":
        rg = torch.zeros(b * P, dtype=torch.int32, device=cuda)
        ex = torch.zeros(b * 2, dtype=torch.uint8, device=cuda)
    else:
        rg = torch.zeros(b * P, dtype=torch.int32).pin_memory()
        ex = torch.zeros(b * 2, dtype=torch.uint8).pin_memory()
    rbase, ebase = rg.data_ptr(), ex.data_ptr()
    stream = torch.cuda.current_stream(cuda)
    srv = s.BurstServer(P) if server else None

    def run(op, bt):
        if srv is not None:
            srv.submit(op, bt)
        elif op == s.BURST_PRE:
            s.preprocess_burst(bt, stream)
        else:
            s.exchange_burst(bt, stream)

    def capture(ids):
        rh = rg.cpu().numpy().view(np.uint32).reshape(b, P)
        eh = ex.cpu().numpy()
        for q in ids:
            sl = q % b
            if q < B:
                assert eh[sl * 2].astype(np.int8) == pe[q], f"exponent of packet {q}"
            if q >= b:
                m = min(P, n - (q - b) * P)
                assert np.array_equal(rh[sl, :m], pp[q, :m].view(np.uint32)), f"payload of packet {q}"

    first = list(range(b))
    run(s.BURST_PRE, s.packet_burst(xd, out, P, W, b, recv, first, [rbase + q * P * 4 for q in first],
                                    [ebase + q * 2 for q in first]))
    torch.cuda.synchronize()
    capture(first)
    # the DPDK timer path re-builds a packet that timed out (ResendPacketCallback
    # -> BuildPacket -> PreprocessSingle(pkt_id), dpdk_worker_thread_utils.inc:
    # 225-265) into a fresh mbuf: the PPP is a pure function of (block, scale),
    # so the resent bytes must equal the outstanding packet's
    if ring == "device":
        spare = torch.zeros(3 * P, dtype=torch.int32, device=cuda)
        spare_x = torch.zeros(6, dtype=torch.uint8, device=cuda)
    else:
        spare = torch.zeros(3 * P, dtype=torch.int32).pin_memory()
        spare_x = torch.zeros(6, dtype=torch.uint8).pin_memory()

    def resend_matches(ids):
        run(s.BURST_PRE, s.packet_burst(xd, out, P, W, b, recv, ids,
                                        [spare.data_ptr() + i * P * 4 for i in range(len(ids))],
                                        [spare_x.data_ptr() + i * 2 for i in range(len(ids))]))
        torch.cuda.synchronize()
        rh = rg.cpu().numpy().view(np.uint32).reshape(b, P)
        sh = spare.cpu().numpy().view(np.uint32).reshape(3, P)
        eh, sx = ex.cpu().numpy(), spare_x.cpu().numpy()
        for i, q in enumerate(ids):
            if q < B:
                assert sx[i * 2] == eh[(q % b) * 2], f"resent exponent of packet {q}"
            if q >= b:
                m = min(P, n - (q - b) * P)
                assert np.array_equal(sh[i, :m], rh[q % b, :m]), f"resent payload of packet {q}"

    pending, received = list(first), 0
    while received < total:
        if pending:
            resend_matches([int(q) for q in rng.choice(pending, size=min(3, len(pending)), replace=False)])
        k = int(rng.integers(0, len(pending) + 1))
        got = []
        for _ in range(k):
            got.append(pending.pop(int(rng.integers(0, len(pending)))))
        if not got:
            continue
        received += len(got)
        bt = s.packet_burst(xd, out, P, W, b, recv, got, [rbase + (q % b) * P * 4 for q in got],
                            [ebase + (q % b) * 2 for q in got], flags=s.FLAG_PROCESS_PACKET)
        run(s.BURST_EXCHANGE, bt)
        torch.cuda.synchronize()
        nxt = [q + b for q in got if q + b < total]
        capture(nxt)
        pending.extend(nxt)
    assert not pending
    if srv is not None:
        srv.close()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref_out.view(np.uint32))


@pytest.mark.gpu
def test_burst_server_idle_restart_and_refusals(cuda):
    """The server leaves its loop after idle_ms without a doorbell and the next
    submit starts another (the burst still completes, bit-exact); a burst with
    another packet size or rounding mode than the server's is refused; close()
    of a server that never ran, and twice, is fine."""
    import time
    import torch
    s = sw()
    P, W, n = 256, 2, 20_000
    x = O.splitmix_normal(17, n)
    xd = torch.from_numpy(x).to(cuda)
    out = torch.zeros(n, device=cuda)
    B = O.num_blocks(n, P)
    b = 16
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    ring = torch.zeros(b * P, dtype=torch.int32).pin_memory()
    extra = torch.zeros(b * 2, dtype=torch.uint8).pin_memory()
    s.BurstServer(P).close()                                   # never started
    srv = s.BurstServer(P, idle_ms=20)
    ids = list(range(b))
    slots = [ring.data_ptr() + q * P * 4 for q in ids]
    exs = [extra.data_ptr() + q * 2 for q in ids]
    srv.submit(s.BURST_PRE, s.packet_burst(xd, out, P, W, b, recv, ids, slots, exs))
    for p0 in range(0, B + b, b):
        time.sleep(0.05)                                       # > idle_ms: the server has left its loop
        got = list(range(p0, min(p0 + b, B + b)))
        srv.submit(s.BURST_EXCHANGE, s.packet_burst(xd, out, P, W, b, recv, got, slots[:len(got)], exs[:len(got)],
                                                    flags=s.FLAG_PROCESS_PACKET))
        if p0 == b:
            srv.stop()                                         # stopped explicitly: restarted by the next submit
    ref = O.dummy_packet_stream(x, P=P, batch_max=b, num_workers=W)[2]
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    with pytest.raises(s.SwitchMLError):                       # another packet size
        srv.submit(s.BURST_PRE, s.packet_burst(xd, out, 64, W, b, recv, [0], slots[:1], exs[:1]))
    with pytest.raises(s.SwitchMLError):                       # another rounding mode
        srv.submit(s.BURST_PRE, s.packet_burst(xd, out, P, W, b, recv, [0], slots[:1], exs[:1],
                                               flags=s.FLAG_ROUND_RNE))
    srv.close()
    srv.close()


@pytest.mark.gpu
def test_burst_server_never_replays_an_unanswered_doorbell(cuda):
    """after a failed submit the doorbell is ahead of `done`; a
    relaunched server must not take that stale doorbell for a new burst.  The
    injected one is an exchange burst on the ring's first window — replayed,
    it would post-process those packets and overwrite their slots with the
    next window's packets, so the real exchange of the same window (and the
    output) would go wrong.  Start the server, give it time to (wrongly)
    replay, then run the slice: bit-exact vs the oracle's packet loop."""
    import time
    import torch
    s = sw()
    P, W, n = 256, 2, 20_000
    x = O.splitmix_normal(19, n)
    xd = torch.from_numpy(x).to(cuda)
    out = torch.zeros(n, device=cuda)
    B = O.num_blocks(n, P)
    b = 16
    recv = torch.zeros(B, dtype=torch.int8, device=cuda)
    ring = torch.zeros(b * P, dtype=torch.int32).pin_memory()
    extra = torch.zeros(b * 2, dtype=torch.uint8).pin_memory()
    srv = s.BurstServer(P, idle_ms=2000)
    ids = list(range(b))
    slots = [ring.data_ptr() + q * P * 4 for q in ids]
    exs = [extra.data_ptr() + q * 2 for q in ids]
    srv.submit(s.BURST_PRE, s.packet_burst(xd, out, P, W, b, recv, ids, slots, exs))
    srv.inject_unanswered(s.BURST_EXCHANGE, s.packet_burst(xd, out, P, W, b, recv, ids, slots, exs,
                                                           flags=s.FLAG_PROCESS_PACKET))
    srv.start()
    time.sleep(0.05)                       # a replaying server would have run the stale burst by now
    for p0 in range(0, B + b, b):
        got = list(range(p0, min(p0 + b, B + b)))
        srv.submit(s.BURST_EXCHANGE, s.packet_burst(xd, out, P, W, b, recv, got, slots[:len(got)], exs[:len(got)],
                                                    flags=s.FLAG_PROCESS_PACKET))
    srv.close()
    ref = O.dummy_packet_stream(x, P=P, batch_max=b, num_workers=W)[2]
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
