"""GPU frame passes against the CPU oracle, through the
C ABI: in-place masking, UTF-8 verdicts, and the fused receive (unmask +
inflate + UTF-8) and send (deflate + mask) paths, on both inflate kernels."""
import random

import numpy as np
import pytest

from beast_amd import synth
from oracle import oracle as O
from tests import utf8_cases
from tests.test_frame import utf8_fuzz

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["lane", "wave"])
def inflate_kernel(request):
    pmd = _pmd()
    assert pmd.lib().bpmd_set_inflate_kernel({"lane": 1, "wave": 2}[request.param]) == 0
    yield request.param
    pmd.lib().bpmd_set_inflate_kernel(0)


def _pmd():
    import torch  # noqa: F401
    from beast_amd import pmd
    return pmd


def _ragged(msgs, rng, fill=0xA5):
    """Messages at random byte alignments with guard bytes between them."""
    offs, pos = [], 0
    for m in msgs:
        pos += rng.randrange(0, 20)
        offs.append(pos)
        pos += len(m)
    buf = bytearray([fill]) * (pos + 64)
    for o, m in zip(offs, msgs):
        buf[o:o + len(m)] = m
    return bytes(buf), offs


def _batch(buf, offs, lens):
    import torch
    pmd = _pmd()
    return pmd.Batch(torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda(),
                     torch.tensor(offs, dtype=torch.int64).cuda(), torch.tensor(lens, dtype=torch.int32).cuda())


def test_mask_matches_oracle_and_leaves_neighbours():
    pmd = _pmd()
    rng = random.Random(5)
    msgs = [rng.randbytes(rng.choice([0, 1, 3, 4, 5, 15, 16, 17, 31, 100, 1000, 4096, 5003])) for _ in range(700)]
    buf, offs = _ragged(msgs, rng)
    keys = [rng.getrandbits(32) for _ in msgs]
    phases = [rng.randrange(4) for _ in msgs]
    b = _batch(buf, offs, [len(m) for m in msgs])
    pmd.mask_batch(b, keys, phases)
    got = b.data.cpu().numpy().tobytes()
    want = bytearray(buf)
    for o, m, k, ph in zip(offs, msgs, keys, phases):
        want[o:o + len(m)] = O.mask(m, k, ph)
    assert got == bytes(want)


def _utf8_corpus(rng):
    msgs = [p for p, _ in utf8_cases.prefixes()]
    msgs += utf8_fuzz(rng, 3000)
    # long texts with one fault placed around 16-byte units and 1 KiB wave steps
    alphabet = ["a", "b", " ", "é", "ж", "語", "\U0001f600", "\n"]
    for _ in range(400):
        s = "".join(rng.choice(alphabet) for _ in range(rng.randrange(50, 3000))).encode()
        k = rng.randrange(5)
        if k == 1:
            s = s[:rng.randrange(len(s))]
        elif k == 2:
            b = bytearray(s)
            at = rng.choice([rng.randrange(len(b)), min(len(b) - 1, 1023), min(len(b) - 1, 15), len(b) - 1])
            b[at] = rng.choice([0x80, 0xbf, 0xc0, 0xc1, 0xe0, 0xed, 0xf0, 0xf4, 0xf5, 0xff, 0x41])
            s = bytes(b)
        msgs.append(s)
    d, _, _ = synth.make_batch("json", [4096] * 8, seed=3)
    msgs += [bytes(d[i * 4096:(i + 1) * 4096]) for i in range(8)]
    return msgs


def test_utf8_matches_oracle():
    pmd = _pmd()
    rng = random.Random(9)
    msgs = _utf8_corpus(rng)
    buf, offs = _ragged(msgs, rng)
    b = _batch(buf, offs, [len(m) for m in msgs])
    res = pmd.utf8_check_batch(b).cpu().numpy()
    want = np.array([O.utf8_check(m) for m in msgs])
    bad = np.nonzero(res != want)[0]
    assert len(bad) == 0, [(msgs[i][:48].hex(), int(res[i]), int(want[i])) for i in bad[:5]]


def _text_corpus(rng, n):
    alphabet = ["a", "{", "\"", ":", " ", "é", "ж", "語", "\U0001f600"]
    msgs, text = [], []
    for i in range(n):
        kind = rng.randrange(4)
        if kind == 0:   # binary
            d, _, _ = synth.make_batch(rng.choice(["binary", "random", "json"]), [rng.choice([0, 7, 900, 4096])],
                                       seed=i)
            msgs.append(bytes(d))
            text.append(0)
            continue
        s = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 2500))).encode()
        if kind == 2 and s:   # not UTF-8
            b = bytearray(s)
            b[rng.randrange(len(b))] = rng.choice([0x80, 0xc0, 0xed, 0xff])
            s = bytes(b)
        elif kind == 3:       # cut inside a code point, maybe
            s = s[:rng.randrange(len(s) + 1)]
        msgs.append(s)
        text.append(1)
    return msgs, text


def test_read_batch_unmasks_inflates_and_checks_text(inflate_kernel):
    pmd = _pmd()
    rng = random.Random(13)
    msgs, text = _text_corpus(rng, 500)
    payloads = [O.pmd_deflate(m, rng.choice([1, 6, 9]), 15, 4) for m in msgs]
    for i in range(0, len(payloads), 37):   # some corrupted payloads too
        q = bytearray(payloads[i])
        if q:
            q[rng.randrange(len(q))] ^= 1 << rng.randrange(8)
        payloads[i] = bytes(q)
    keys = [rng.getrandbits(32) for _ in msgs]
    masked = [O.mask(p, k) for p, k in zip(payloads, keys)]
    buf, offs = _ragged(masked, rng)
    src = _batch(buf, offs, [len(p) for p in masked])
    caps = [max(len(m), 1) for m in msgs]
    import torch
    res = pmd.read_batch(src, torch.tensor(caps, dtype=torch.int32), key=keys, text=text)
    torch.cuda.synchronize()
    st = res.status.cpu().numpy()
    outs = res.out.to_host()
    assert src.data.cpu().numpy().tobytes() == buf   # input untouched
    for i, p in enumerate(payloads):
        est, eout = O.pmd_inflate(p, cap=caps[i])
        if est == 0 and text[i] and O.utf8_check(eout) != 0:
            est = pmd.BAD_FRAME_PAYLOAD
        assert int(st[i]) == est, (i, int(st[i]), est)
        assert outs[i] == eout, i


def test_read_batch_without_key_or_text_is_inflate(inflate_kernel):
    pmd = _pmd()
    rng = random.Random(14)
    msgs, _ = _text_corpus(rng, 200)
    payloads = [O.pmd_deflate(m, 6, 15, 4) for m in msgs]
    src = pmd.Batch.from_host(payloads)
    a = pmd.read_batch(src, 3000)
    b = pmd.inflate_batch(src, 3000)
    assert a.status.cpu().tolist() == b.status.cpu().tolist()
    assert a.out.to_host() == b.out.to_host()


def test_write_batch_masks_the_deflate_payloads():
    pmd = _pmd()
    rng = random.Random(15)
    msgs = []
    for i in range(300):
        d, _, _ = synth.make_batch(rng.choice(["json", "corpus1", "binary", "zeros"]),
                                   [rng.choice([0, 1, 100, 4095, 4096, 5000, 20000])], seed=i)
        msgs.append(bytes(d))
    keys = [rng.getrandbits(32) for _ in msgs]
    src = pmd.Batch.from_host(msgs)
    plain = pmd.deflate_batch(src, level=6)
    masked = pmd.write_batch(src, key=keys, level=6)
    assert masked.status.cpu().tolist() == plain.status.cpu().tolist()
    pl, ms = plain.out.to_host(), masked.out.to_host()
    for i in range(len(msgs)):
        assert O.mask(ms[i], keys[i]) == pl[i], i
        st, out = O.pmd_inflate(pl[i], cap=max(len(msgs[i]), 1))
        assert st == 0 and out == msgs[i]


@pytest.mark.parametrize("frame_max", [125, 126, 4096, 65536, 1 << 20])
def test_frame_batch_matches_oracle(frame_max):
    """bpmd_frame_batch's wire bytes equal the oracle's frame loop
    (write.hpp:463-545, frame.hpp:134-175), masked and unmasked, with
    per-message opcodes and RSV1 flags, ragged lengths and 7/16/64-bit
    frame lengths."""
    import torch
    pmd = _pmd()
    rng = random.Random(17 + frame_max)
    lens = [0, 1, 3, 15, 16, 17, 125, 126, 127, 4095, 4096, 4097, 65535, 65536, 70001] + \
        [rng.randrange(0, 9000) for _ in range(150)]
    msgs = [rng.randbytes(n) for n in lens]
    ops = [rng.choice([1, 2]) for _ in msgs]
    comp = [rng.choice([0, 1]) for _ in msgs]
    src = pmd.Batch.from_host(msgs)
    for masked in (False, True):
        cnt = pmd.frame_counts(src.len, frame_max).tolist()
        keys = [rng.getrandbits(32) for _ in range(sum(cnt))] if masked else None
        wire = pmd.frame_batch(src, frame_max, op=torch.tensor(ops, dtype=torch.uint8),
                               compressed=torch.tensor(comp, dtype=torch.uint8), keys=keys)
        torch.cuda.synchronize()
        got = wire.to_host()
        k0 = 0
        for i, m in enumerate(msgs):
            ks = keys[k0:k0 + cnt[i]] if masked else None
            k0 += cnt[i]
            assert got[i] == O.frame_write(m, ops[i], bool(comp[i]), keys=ks, frame_max=frame_max), (i, masked)


def test_write_then_frame_round_trip():
    """Send path end to end: GPU deflate, GPU framing with client keys; the
    frames parsed and unmasked on the host give back the payloads, and the
    payloads inflate (oracle) to the messages."""
    import torch
    pmd = _pmd()
    rng = random.Random(18)
    msgs = []
    for i in range(200):
        d, _, _ = synth.make_batch(rng.choice(["json", "binary"]), [rng.choice([0, 10, 4096, 9000, 30000])], seed=i)
        msgs.append(bytes(d))
    src = pmd.Batch.from_host(msgs)
    payloads = pmd.deflate_batch(src, level=6)
    assert payloads.status.cpu().tolist() == [0] * len(msgs)
    pb = payloads.out
    cnt = pmd.frame_counts(pb.len, 4096).tolist()
    keys = [rng.getrandbits(32) for _ in range(sum(cnt))]
    wire = pmd.frame_batch(pb, 4096, op=1, compressed=True, keys=keys).to_host()
    torch.cuda.synchronize()
    k0 = 0
    for i, w in enumerate(wire):
        # parse: header, key, unmask, concatenate
        pos, out, first = 0, b"", True
        while True:
            b0, b1 = w[pos], w[pos + 1]
            assert (b0 & 0x0F) == (1 if first else 0) and bool(b0 & 0x40) == first and b1 & 0x80
            ln, pos = b1 & 0x7F, pos + 2
            if ln == 126:
                ln, pos = int.from_bytes(w[pos:pos + 2], "big"), pos + 2
            elif ln == 127:
                ln, pos = int.from_bytes(w[pos:pos + 8], "big"), pos + 8
            key = int.from_bytes(w[pos:pos + 4], "little")
            assert key == keys[k0]
            k0, pos = k0 + 1, pos + 4
            out += O.mask(w[pos:pos + ln], key)
            pos += ln
            first = False
            if b0 & 0x80:
                break
        assert pos == len(w)
        st, plain = O.pmd_inflate(out, cap=max(len(msgs[i]), 1))
        assert st == 0 and plain == msgs[i], i
