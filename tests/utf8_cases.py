"""The expectations of the reference's own UTF-8 tests
(test/beast/websocket/utf8_checker.cpp), restated as data.

Each case is (segments, expected write() result per segment, expected
finish() result or None when the reference test does not call finish()).
Line numbers cite the reference test the case comes from.
"""


def cases():
    out = []

    def add(segs, writes, fin=None):
        out.append(([bytes(s) for s in segs], list(writes), fin))

    # testOneByteSequence (:27-81)
    for c in range(128):
        add([[c]], [True], True)
    for c in range(128, 192):
        add([[c]], [False])
    for c in range(192, 224):
        if c < 194:
            add([[c]], [False])
        else:
            add([[c]], [True], False)
    for c in range(224, 240):
        add([[c]], [True], False)
    for c in range(240, 245):
        add([[c]], [True], False)
    for c in range(245, 256):
        add([[c]], [False])

    # testTwoByteSequence (:84-128)
    add([[0xc1, 0xbf]], [False])
    for i in (194, 223):
        for j in (128, 191):
            add([[i, j]], [True], True)
        for j in (0, 127, 192, 255):
            add([[i, j]], [False])
        add([[i], [255]], [True, False])

    # testThreeByteSequence (:131-276); 237 is not among the tested leads
    add([[0xef, 0xbf, 0xbf]], [True], True)
    for i in (224, 239):
        b = 160 if i == 224 else 128
        e = 191
        for j in (b, e):
            for k in (128, 191):
                add([[i, j, k]], [True], True)
                if i == 224:
                    add([[i]], [True], False)
                else:
                    add([[i], [j, k]], [True, True])
                add([[i, j], [k]], [True, True])
                if i == 224:
                    for l in (0, 159, 192, 255):
                        add([[i, l, k]], [False])
                        add([[i, l]], [False])
            for k in (0, 127, 192, 255):
                add([[i, j, k]], [False])
            add([[i, j], [255]], [True, False])
        for j in (0, b - 1, e + 1, 255):
            add([[i, j, 255]], [False])
        if i == 224:
            add([[i]], [True], False)
        else:
            add([[i], [255]], [True, False])

    # testFourByteSequence (:279-429)
    for i in (240, 244):
        b = 144 if i == 240 else 128
        e = 143 if i == 244 else 191
        bad2 = (0, 143, 192, 255) if i == 240 else (0, 127, 144, 255)
        for j in range(b, e + 1):
            for k in (128, 191):
                for n in (128, 191):
                    add([[i, j, k, n]], [True], True)
                    add([[i], [j, k, n]], [True, True])
                    add([[i, j], [k, n]], [True, True])
                    add([[i, j, k], [n]], [True, True])
                    for r in bad2:
                        add([[i, r, k, n]], [False])
                        add([[i, r]], [False])
                for r in (0, 127, 192, 255):
                    add([[i, j, k, r]], [False])
                add([[i, j, k], [255]], [True, False])
            for r in (0, 127, 192, 255):
                add([[i, j, r, 255]], [False])
            add([[i, j], [255]], [True, False])
        for r in (0, b - 1, e + 1, 255):
            add([[i, r, 255, 255]], [False])
        add([[i], [255]], [True, False])
    for r in (245, 255):
        add([[r, 255, 255, 255]], [False])

    # testWithStreamBuffer (:432-479): valid texts, fed 3 bytes at a time
    texts = [
        "48 65 69 7A C3 B6 6C 72 C3 BC 63 6B 73 74 6F C3 9F 61 62 64 C3 A4 6D 70 66 75 6E 67",
        "CE 93 CE B1 CE B6 CE AD CE B5 CF 82 20 CE BA CE B1 E1 BD B6 20 CE BC CF 85 CF 81 CF 84 CE B9 E1 BD B2 "
        "CF 82 20 CE B4 E1 BD B2 CE BD 20 CE B8 E1 BD B0 20 CE B2 CF 81 E1 BF B6 20 CF 80 CE B9 E1 BD B0 20 CF 83 "
        "CF 84 E1 BD B8 20 CF 87 CF 81 CF 85 CF 83 CE B1 CF 86 E1 BD B6 20 CE BE CE AD CF 86 CF 89 CF 84 CE BF",
        "C3 81 72 76 C3 AD 7A 74 C5 B1 72 C5 91 20 74 C3 BC 6B C3 B6 72 66 C3 BA 72 C3 B3 67 C3 A9 70",
        "F0 90 80 80",
    ]
    for t in texts:
        d = bytes.fromhex(t)
        segs = [d[o:o + 3] for o in range(0, len(d), 3)]
        add(segs, [True] * len(segs), True)

    # testBranches (:482-520)
    add([b"\xc2\x80" * 15], [True], True)
    add([b"********\x80***"], [False])

    # AutodeskTests (:523-544)
    add([b"start\xe0", b"\xa6\x81end"], [True, True], True)

    # Autobahn 6.4.2 and 6.4.4 (:579-588)
    head = bytes([0xCE, 0xBA, 0xE1, 0xBD, 0xB9, 0xCF, 0x83, 0xCE, 0xBC, 0xCE, 0xB5, 0xF4])
    add([head, b"\x90", bytes([0x80, 0x80, 0x65, 0x64, 0x69, 0x74, 0x65, 0x64])], [True, False, False])
    add([head, b"\x90"], [True, False])
    return out


def prefixes():
    """(bytes, verdict) for every prefix the cases feed: 2 where that write()
    fails, else 0 / 1 by the case's finish() when it is the last segment and
    the reference checks it, else None (write() ok, finish() unchecked)."""
    res = []
    for segs, writes, fin in cases():
        acc = b""
        for k, s in enumerate(segs):
            acc += s
            if not writes[k]:
                res.append((acc, 2))
            elif k == len(segs) - 1 and fin is not None:
                res.append((acc, 0 if fin else 1))
            else:
                res.append((acc, None))
    return res
