"""CPU check of the per-stream inflate kernel's own logic
(beast_amd/csrc/pmd_zstream.hip, zstream_run), compiled for the host by
tests/model/zstream_host.py: every write()'s status, z_params and output
bytes must equal the oracle's restatement of Beast's inflate_stream.  The
GPU build of the same code runs the same cases in tests/test_gpu_zstream.py."""
import pytest

from tests import zstream_cases as Z
from tests.model import zstream_host as H


def make(wbits):
    return H.HostInflater(wbits)


@pytest.mark.parametrize("kind", ["json", "binary", "random"])
@pytest.mark.parametrize("level,mem", [(1, 4), (6, 4), (9, 9), (6, 1)])
def test_connection_random_cuts(kind, level, mem):
    Z.case_connection_random_cuts(make, kind, level, mem)


def test_foreign_encoder_connection():
    Z.case_foreign_payloads(make)


@pytest.mark.parametrize("hpar", ["1", "0"])
def test_code_length_loops(hpar, monkeypatch):
    """The dynamic header's code lengths: hdr_par's windows (default) and the
    serial loop (BPMD_ZSTREAM_HPAR=0) against the oracle, under random cuts,
    input a byte at a time, the KATs and corrupted headers."""
    monkeypatch.setenv("BPMD_ZSTREAM_HPAR", hpar)
    Z.case_connection_random_cuts(make, "json", 8, 4)
    Z.case_byte_at_a_time_input(make)
    Z.case_kat_split(make, every_cut=False)
    Z.case_errors(make)


def test_output_room_one_byte():
    Z.case_output_room_one_byte(make, n_calls=1500)


def test_byte_at_a_time_input():
    Z.case_byte_at_a_time_input(make)


def test_flush_mix():
    Z.case_flush_mix(make)


def test_flush_trees_kat():
    Z.case_flush_trees_kat(make)


def test_kat_split():
    Z.case_kat_split(make)


def test_small_window():
    Z.case_small_window(make)


def test_end_of_stream():
    Z.case_end_of_stream(make)


def test_stored_blocks():
    Z.case_stored_blocks(make)


def test_errors():
    Z.case_errors(make)


def test_issue3028_one_byte_reads():
    msg = Z.issue3028_message()
    from oracle import oracle as O
    pays = O.pmd_deflate_stream([msg] * 3, 8, 15, 4)
    res = Z.ws_replay(make, [[p] for p in pays], size=1)
    assert all(r == (msg, 0) for r in res)


def test_issue1630_packets():
    from oracle import oracle as O
    frames = Z.issue1630_frames()
    res = Z.ws_replay(make, [[p] for _, p in frames], size=4096)
    for got, st in res:
        assert st == 0 and O.utf8_check(got) == 0
