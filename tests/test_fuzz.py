"""CPU sanitizer fuzzing of libfsm's host parsers (the parsers take
untrusted text and had no ASan/UBSan build).

tests/fuzz/Makefile compiles flatten.cpp (SPADE.scala:145-212, TSR.scala:109-143
parsing of SPMF lines and token streams), ingest.cpp (util/SPMFBuilder.scala
formats) and results.cpp (result documents, rule queries) unchanged with g++
-fsanitize=address,undefined -fno-sanitize-recover=all into
tests/fuzz/parsers_harness.  Hypothesis generates malformed and well-formed
inputs; the harness must exit 0 with one "ok" / "err <code>" line per case:
bad input comes back as an fsm error code, never as a sanitizer abort.
No GPU is involved."""
import os
import struct
import subprocess

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

HERE = os.path.dirname(os.path.abspath(__file__))
FUZZ = os.path.join(HERE, "fuzz")
BIN = os.path.join(FUZZ, "build", "parsers_harness")


@pytest.fixture(scope="module")
def harness():
    subprocess.run(["make", "-s", "-C", FUZZ], check=True)
    return BIN


def case(kind, payload):
    return struct.pack("<BI", kind, len(payload)) + payload


def lines_payload(recs):
    b = struct.pack("<I", len(recs))
    for sid, line in recs:
        raw = line.encode("utf-8", "surrogatepass") if isinstance(line, str) else line
        b += struct.pack("<iI", sid, len(raw)) + raw
    return b


def tokens_payload(seqs):
    b = struct.pack("<I", len(seqs))
    for sid, toks in seqs:
        b += struct.pack("<iI", sid, len(toks)) + struct.pack("<%dq" % len(toks), *toks)
    return b


def run(harness, blob, ncases):
    p = subprocess.run([harness], input=blob, capture_output=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    out = p.stdout.decode().splitlines()
    assert len(out) == ncases and all(l.split()[1] in ("ok", "err") for l in out), out[-3:]
    return out


# SPMF-ish tokens: items, separators, timestamps, junk, odd spacing
tok = st.one_of(st.integers(-3, 40).map(str), st.sampled_from(["-1", "-2", "<3>", "<", ">", "<-1>", "<x>", "",
                                                                "2147483648", "-2147483649", "+5", "1e3",
                                                                "99999999999999999999", "é", "\x00"]),
                st.text(max_size=4))
line = st.one_of(st.lists(tok, max_size=12).map(" ".join), st.text(max_size=30),
                 st.binary(max_size=30).map(lambda b: b.decode("latin-1")))
recs = st.lists(st.tuples(st.integers(-2, 6), line), max_size=8)
seqs = st.lists(st.tuples(st.integers(-2, 6), st.lists(st.one_of(st.integers(-3, 50),
                                                                  st.integers(-(1 << 63), (1 << 63) - 1)),
                                                        max_size=20)), max_size=8)
files = st.one_of(st.text(alphabet="0123456789 ,;|-\n\r\t<>abc", max_size=200), st.binary(max_size=200).map(
    lambda b: b.decode("latin-1")))


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.tuples(st.integers(0, 3), recs, seqs), min_size=1, max_size=12))
def test_flatten_lines_and_tokens_under_sanitizers(harness, cases):
    blob = b""
    for kind, r, q in cases:
        blob += case(kind, lines_payload(r) if kind < 2 else tokens_payload(q))
    run(harness, blob, len(cases))


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.tuples(st.integers(-1, 6), st.integers(-2, 5), files), min_size=1, max_size=12))
def test_ingest_formats_under_sanitizers(harness, cases):
    blob = b""
    for fmt, limit, text in cases:
        blob += case(4, struct.pack("<iq", fmt, limit) + text.encode("utf-8", "surrogatepass"))
    run(harness, blob, len(cases))


@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.tuples(st.integers(0, 40), st.lists(st.integers(-(1 << 31), (1 << 31) - 1), max_size=60)),
                min_size=1, max_size=8))
def test_result_documents_under_sanitizers(harness, cases):
    blob = b""
    for n, ints in cases:
        blob += case(5, struct.pack("<I", n) + struct.pack("<%di" % len(ints), *ints))
    run(harness, blob, len(cases))


def test_harness_reports_parse_errors(harness):
    """The harness sees the parsers' verdicts: a well-formed line parses, an
    empty token (double space, SPADE.scala:161) is FSM_EPARSE."""
    blob = case(0, lines_payload([(0, "1 2 -1 3 -1 -2")])) + case(0, lines_payload([(0, "1  2 -1")])) + \
        case(4, struct.pack("<iq", 4, -1) + b"1 2 3\n4 5\n")
    out = run(harness, blob, 3)
    assert out[0] == "0 ok 0" and out[1].startswith("0 err 2") and out[2] == "4 ok 0"
