"""Generates tests/golden/cve_2018_25032.json: the two inputs of the
reference's CVE-2018-25032 deflate test (test/beast/zlib/deflate_stream.cpp:
610-636, fixtures/CVE_2018_25032/{default,fixed}.hpp), decoded from their C
string literals to bytes.  The fixture is data only.  Usage:
    python tests/golden/make_cve_2018_25032.py [/root/reference]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_ws_issues import c_literals  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main(ref="/root/reference"):
    d = os.path.join(ref, "test", "beast", "zlib", "fixtures", "CVE_2018_25032")
    doc = {"source": "test/beast/zlib/fixtures/CVE_2018_25032/{default,fixed}.hpp",
           "test": "test/beast/zlib/deflate_stream.cpp:610-636",
           # testCVE(input, level, strategy): (fixture, level, strategy) rows of :628-635
           "cases": [["default", 1, "fixed"], ["default", 2, "fixed"], ["default", 6, "fixed"],
                     ["fixed", 1, "normal"], ["fixed", 2, "normal"], ["fixed", 6, "normal"]]}
    for name in ("default", "fixed"):
        txt = open(os.path.join(d, name + ".hpp"), encoding="latin-1").read()
        data = c_literals(txt[txt.index("="):])
        assert b"\0" not in data   # strlen() is the length the test uses
        doc[name] = data.decode("ascii")
    with open(os.path.join(HERE, "cve_2018_25032.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print({k: len(doc[k]) for k in ("default", "fixed")})


if __name__ == "__main__":
    main(*sys.argv[1:])
