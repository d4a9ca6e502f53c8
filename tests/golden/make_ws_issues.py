"""Generates tests/golden/ws_issues.json: the input data of two of the
reference's websocket read-path regression tests, as bytes (hex).

* issue 1630 (test/beast/websocket/read3.cpp:619-1009): four packets of
  compressed text frames (server to client, unmasked, context takeover) whose
  deflate blocks split multi-byte UTF-8 characters across calls;
* issue 3028 (read3.cpp:1133-1226): the text message a client writes three
  times while the server reads it back one byte per read_some.

Run with the reference present (/root/reference); the fixture is data only
(the C string literals of those tests decoded to bytes).  Usage:
    python tests/golden/make_ws_issues.py [/root/reference]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def c_literals(text: str) -> bytes:
    """Concatenates the C string literals in `text` and decodes escapes."""
    out = bytearray()
    for lit in re.findall(r'"((?:[^"\\]|\\.)*)"', text, flags=re.S):
        i = 0
        while i < len(lit):
            c = lit[i]
            if c != "\\":
                out += c.encode("latin-1")
                i += 1
                continue
            e = lit[i + 1]
            if e == "x":   # greedy hex digits, as C does
                j = i + 2
                while j < len(lit) and lit[j] in "0123456789abcdefABCDEF":
                    j += 1
                v = int(lit[i + 2:j], 16)
                assert v < 256
                out.append(v)
                i = j
            elif e in "01234567":
                j = i + 1
                while j < len(lit) and j < i + 4 and lit[j] in "01234567":
                    j += 1
                out.append(int(lit[i + 1:j], 8))
                i = j
            else:
                out += {"n": b"\n", "r": b"\r", "t": b"\t", "0": b"\0", "\\": b"\\", '"': b'"', "'": b"'"}[e]
                i += 2
    return bytes(out)


def sbuf_args(body: str):
    """The argument text of every sbuf( ... ) call in `body`."""
    res = []
    for m in re.finditer(r"sbuf\(", body):
        depth, i = 1, m.end()
        in_str = False
        while depth:
            c = body[i]
            if in_str:
                if c == "\\":
                    i += 1
                elif c == '"':
                    in_str = False
            elif c == '"':
                in_str = True
            elif c == "(":
                depth += 1
            elif c == ")":
                depth -= 1
            i += 1
        res.append(body[m.end():i - 1])
    return res


def function_body(src: str, name: str) -> str:
    at = src.index(name + "()")
    start = src.index("{", at)
    depth, i = 0, start
    while True:
        if src[i] == "{":
            depth += 1
        elif src[i] == "}":
            depth -= 1
            if depth == 0:
                return src[start:i + 1]
        i += 1


def main(ref="/root/reference"):
    path = os.path.join(ref, "test", "beast", "websocket", "read3.cpp")
    src = open(path, encoding="latin-1").read()
    b1630 = function_body(src, "testIssue1630")
    packets = [c_literals(a) for a in sbuf_args(b1630[b1630.index("packets[]"):])]
    b3028 = function_body(src, "testIssue3028")
    msg = c_literals(sbuf_args(b3028)[0])
    doc = {
        "source": "test/beast/websocket/read3.cpp (testIssue1630, testIssue3028)",
        "issue1630": {"packets_hex": [p.hex() for p in packets]},
        "issue3028": {"message_hex": msg.hex(), "reads": 3, "read_size": 1},
    }
    with open(os.path.join(HERE, "ws_issues.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print("packets", [len(p) for p in packets], "message", len(msg))


if __name__ == "__main__":
    main(*sys.argv[1:])
