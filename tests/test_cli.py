"""The `sahara` CLI (bin/sahara): flags, stdout blocks, output format and exit
codes of src/sahara/index.cpp and src/sahara/search.cpp, over the golden
fixtures. Error paths that fail before the device is touched run on CPU."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import hits_as_rows
from test_golden import CASES, GOLD, IDX, expected, limit_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAHARA = os.environ.get("SAHARA_CLI") or os.path.join(ROOT, "bin", "sahara")  # SAHARA_CLI: e.g. bin/sahara_asan


def run(*args, cwd=None):
    if not os.path.exists(SAHARA):
        pytest.fail("bin/sahara missing: run `make` (or __graft_entry__.build())")
    p = subprocess.run([SAHARA, *map(str, args)], capture_output=True, text=True, cwd=cwd, timeout=300)
    return p.returncode, p.stdout, p.stderr


def write(path, text):
    path.write_text(text)
    return path


def test_list_generators():
    rc, out, _ = run("search_scheme", "list-generators")
    assert rc == 0
    names = [line.split(" - ")[0].strip() for line in out.splitlines()]
    assert {"backtracking", "pigeon", "h2-k1", "h2-k2", "h2-k3"} <= set(names)


def test_no_command_is_an_error():
    assert run()[0] == 1
    assert run("frobnicate")[0] == 1


def test_index_rejects_invalid_character(tmp_path):
    fa = write(tmp_path / "r.fa", ">r1 first\nACGTACGTNNAC\n>r2\nACGXTT\n")
    rc, out, err = run("index", fa)
    assert rc == 1
    assert out.startswith(f"constructing an index for {fa}\n")
    assert "ref 'r2' (2) has invalid character 'X' (0x58) at position 3" in err
    assert not (tmp_path / "r.fa.idx").exists()


def test_index_dna4_rejects_n(tmp_path):
    fa = write(tmp_path / "r.fa", ">r1\nACGTNACG\n")
    rc, _, err = run("index", fa, "--dna4")
    assert rc == 1 and "invalid character 'N' (0x4e) at position 4" in err


def test_index_empty_reference(tmp_path):
    fa = write(tmp_path / "r.fa", "")
    rc, _, err = run("index", fa)
    assert rc == 1 and "was empty - abort" in err


def test_search_requires_query_and_index(tmp_path):
    assert run("search", "-i", os.path.join(GOLD, IDX["a"]))[0] == 1
    assert run("search", "-q", os.path.join(GOLD, "reads_a.fa"))[0] == 1


def test_search_missing_index(tmp_path):
    rc, _, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", tmp_path / "nope.idx")
    assert rc == 1 and "no valid index path at" in err


def test_search_unknown_sigma(tmp_path):
    bad = tmp_path / "x.idx"
    bad.write_bytes((7).to_bytes(8, "little") + b"\0" * 64)
    rc, _, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", bad)
    assert rc == 1 and "unknown index with 7 letters" in err


def test_search_invalid_query_character(tmp_path):
    q = write(tmp_path / "q.fa", ">q1\nACGTACGT\n>q2\nACGTAXGT\n")
    rc, _, err = run("search", "-q", q, "-i", os.path.join(GOLD, IDX["a"]))
    assert rc == 1
    assert "query 'q2' (3) has invalid character at position 5 'X'(58)" in err


def test_index_crlf_multiline_records_count_positions_in_sequence(tmp_path):
    """The parallel ingest (fasta.h parseFastaParallel) reads records across
    lines and CRLF breaks like ivio's reader: positions count sequence
    characters only, and the header keeps its text after '>'."""
    fa = write(tmp_path / "r.fa", ">r1\r\nACGT\r\nACGT\r\n>r2 x>y\r\nAC\r\n\r\nGTXA\r\n")
    rc, _, err = run("index", fa)
    assert rc == 1 and "ref 'r2 x>y' (2) has invalid character 'X' (0x58) at position 4" in err


def test_fasta_sequence_before_header_is_an_error(tmp_path):
    fa = write(tmp_path / "r.fa", "ACGT\n>r1\nACGT\n")
    rc, _, err = run("index", fa)
    assert rc == 1 and "malformed FASTA" in err


def test_search_invalid_query_numbering_without_reverse(tmp_path):
    q = write(tmp_path / "q.fa", ">q1\nACGTACGT\n>q2\nACGTAXGT\n")
    rc, _, err = run("search", "-q", q, "-i", os.path.join(GOLD, IDX["a"]), "--no-reverse")
    assert rc == 1 and "query 'q2' (2) has invalid character at position 5 'X'(58)" in err


def test_search_empty_queries(tmp_path):
    q = write(tmp_path / "q.fa", "")
    rc, _, err = run("search", "-q", q, "-i", os.path.join(GOLD, IDX["a"]))
    assert rc == 1 and "was empty - abort" in err


def test_search_bad_enum_values():
    base = ["search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"])]
    assert run(*base, "-m", "fast")[0] == 1
    assert run(*base, "-d", "hamming")[0] == 1


# ------------------------------------------------------------------ GPU ----

def cli_args(c):
    a = ["-e", c["k"], "-g", c["generator"], "-d", c["metric"], "-m", c["mode"]]
    if not c["reverse"]:
        a.append("--no-reverse")
    return a


def read_hits(path, cols):
    a = np.loadtxt(path, dtype=np.uint64, ndmin=2)
    return a.reshape(-1, cols)


@pytest.mark.gpu
@pytest.mark.parametrize("fixture,extra,name", [("a", [], "ref_a.fa.idx"), ("b", ["--dna4"], "ref_b.fa.dna4.idx")])
def test_cli_index_writes_golden_bytes(fixture, extra, name, tmp_path, gpu_device):
    fa = tmp_path / f"ref_{fixture}.fa"
    shutil.copy(os.path.join(GOLD, f"ref_{fixture}.fa"), fa)
    rc, out, err = run("index", fa, *extra)
    assert rc == 0, err
    assert "  references: " in out and "  index creation time:" in out and "  total time:" in out
    assert (tmp_path / name).read_bytes() == open(os.path.join(GOLD, name), "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_cli_search_matches_golden(name, tmp_path, gpu_device):
    c = CASES[name]
    out = tmp_path / "hits.txt"
    rc, so, err = run("search", "-q", os.path.join(GOLD, f"reads_{c['fixture']}.fa"),
                      "-i", os.path.join(GOLD, IDX[c["fixture"]]), "-o", out, "--emit-errors", *cli_args(c))
    assert rc == 0, err
    assert np.array_equal(hits_as_rows(read_hits(out, 4)), expected(name))
    assert f"  number of hits:      {c['hits']:>10}" in so
    fwd = c["patterns"] // (2 if c["reverse"] else 1)
    assert f"fwd queries: {fwd}\nbwd queries: {c['patterns'] - fwd}\n" in so
    assert sum(line.startswith("node count: ") for line in so.splitlines()) == (c["k"] + 1 if c["mode"] == "besthits" else 1)


@pytest.mark.gpu
def test_cli_default_output_format(tmp_path, gpu_device):
    rc, so, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                      "-e", 2, cwd=tmp_path)
    assert rc == 0, err
    rows = read_hits(tmp_path / "sahara-output.txt", 3)      # "qid seqId pos" (search.cpp:258)
    want = expected("a_lev_k2")[:, :3]
    assert np.array_equal(rows[np.lexsort(rows.T[::-1])], want[np.lexsort(want.T[::-1])])
    for line in ("config:", "  query:               ", "  generator:           h2-k2",
                 "  allowed errors:      2", "  reverse complements: true", "  search mode:         all",
                 "  max hits:            0", "  output path:         sahara-output.txt", "stats:",
                 "  ld queries time:", "  ld index time:", "  searchScheme time:", "  search time:",
                 "  locate time:", "  result time:", "  total time:", "  queries per second:"):
        assert line in so, line


@pytest.mark.gpu
def test_cli_limit_queries_and_max_hits(tmp_path, gpu_device):
    out = tmp_path / "h.txt"
    rc, so, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                      "-e", 2, "--limit_queries", 33, "--max_hits", 2, "--emit-errors", "-o", out)
    assert rc == 0, err
    want = expected("a_lev_k2")
    want = limit_rows(want[want[:, 0] < 33], 2)
    assert np.array_equal(hits_as_rows(read_hits(out, 4)), want)
    assert "fwd queries: 16\nbwd queries: 17\n" in so


@pytest.mark.gpu
def test_cli_crlf_wrapped_queries_equal_golden(tmp_path, gpu_device):
    """The same reads as CRLF records wrapped at 7 columns: the same hits."""
    recs = []
    for line in open(os.path.join(GOLD, "reads_a.fa")):
        line = line.rstrip("\n")
        if line.startswith(">"):
            recs.append([line, ""])
        else:
            recs[-1][1] += line
    text = "".join(h + "\r\n" + "".join(s[i:i + 7] + "\r\n" for i in range(0, len(s), 7)) for h, s in recs)
    q = write(tmp_path / "q.fa", text)
    out = tmp_path / "h.txt"
    rc, _, err = run("search", "-q", q, "-i", os.path.join(GOLD, IDX["a"]), "-e", 2, "--emit-errors", "-o", out)
    assert rc == 0, err
    assert np.array_equal(hits_as_rows(read_hits(out, 4)), expected("a_lev_k2"))


@pytest.mark.gpu
def test_cli_fm_only_mode(tmp_path, gpu_device):
    out = tmp_path / "h.txt"
    rc, _, err = run("search", "-q", os.path.join(GOLD, "reads_b.fa"), "-i", os.path.join(GOLD, IDX["b"]),
                     "-e", 3, "-g", "h2-k3", "--fm-only", "--emit-errors", "-o", out)
    assert rc == 0, err
    assert np.array_equal(hits_as_rows(read_hits(out, 4)), expected("b_lev_k3"))


@pytest.mark.gpu
def test_cli_errors_after_index_load(tmp_path, gpu_device):
    q = write(tmp_path / "q.fa", ">q1\nACGTACGTAC\n>q2\nACGTAC\n")
    rc, _, err = run("search", "-q", q, "-i", os.path.join(GOLD, IDX["a"]))
    assert rc == 1 and "must have the length of the first" in err
    rc, _, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                     "-g", "nope")
    assert rc == 1 and 'unknown search scheme generetaror "nope"' in err
    # names the reference lists whose tables are not restated here keep its error
    for name in ("optimum", "01*0_opt", "hato"):
        rc, _, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                         "-g", name)
        assert rc == 1 and f'unknown search scheme generetaror "{name}"' in err and "pex-bu-l" in err


@pytest.mark.gpu
@pytest.mark.parametrize("gen", ["kianfar", "pex-td", "pex-td-l", "pex-bu", "pex-bu-l"])
def test_cli_new_generators_find_the_golden_positions(tmp_path, gpu_device, gen):
    """-g with the PEX and Kianfar schemes: the same (qid, seqId, pos) set as
    the golden file of the default generator (a complete scheme finds every
    position; duplicates and e follow the scheme)."""
    out = tmp_path / "h.txt"
    rc, _, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                     "-e", 2, "-g", gen, "-o", out)
    assert rc == 0, err
    got = {tuple(r) for r in read_hits(out, 3).tolist()}
    want = {tuple(r[:3]) for r in expected("a_lev_k2").tolist()}
    assert got == want


# ------------------------------------------------------- read_simulator ----

def parse_sim(path):
    recs, head = [], None
    for line in open(path):
        line = line.rstrip("\n")
        if line.startswith(">"):
            head = line[1:]
            recs.append([head, ""])
        else:
            recs[-1][1] += line
    return recs


def apply_transcript(ref, pos, trans, read):
    """The read_simulator.cpp:204-231 semantics, checked against its output."""
    p = j = 0
    for t in trans:
        if t == "M":
            assert read[j] == ref[pos + p]
            p += 1
            j += 1
        elif t == "S":
            assert read[j] != ref[pos + p]
            p += 1
            j += 1
        elif t == "I":
            j += 1
        elif t == "D":
            p += 1
    assert j == len(read)


def test_read_simulator_transcripts_and_determinism(tmp_path):
    ref = os.path.join(GOLD, "ref_b.fa")  # ACGT only
    seq = "".join(l.strip() for l in open(ref) if not l.startswith(">"))
    args = ["read_simulator", "-i", ref, "-l", 60, "-n", 50, "-e", 3, "--seed", 5, "--fasta_line_length", 25]
    rc, out, err = run(*args, "-o", tmp_path / "a.fa")
    assert rc == 0, err
    assert out == "loaded fasta file - start simulating\n"
    assert run(*args, "-o", tmp_path / "b.fa")[0] == 0
    assert (tmp_path / "a.fa").read_bytes() == (tmp_path / "b.fa").read_bytes()
    lines = open(tmp_path / "a.fa").read().splitlines()
    assert all(len(l) <= 25 for l in lines if not l.startswith(">"))
    recs = parse_sim(tmp_path / "a.fa")
    assert len(recs) == 50
    for i, (head, read) in enumerate(recs):
        m = __import__("re").fullmatch(r"simulated-(\d+) \(seqid:(\d+), pos:(\d+), trans:([MSID]+)\)", head)
        assert m and int(m.group(1)) == i and int(m.group(2)) == 0
        trans = m.group(4)
        assert len(read) == 60 and sum(c != "M" for c in trans) == 3
        apply_transcript(seq, int(m.group(3)), trans, read)
    rc, _, _ = run("read_simulator", "-i", ref, "-l", 60, "-n", 50, "-e", 3, "--seed", 6, "-o", tmp_path / "c.fa")
    assert rc == 0 and (tmp_path / "c.fa").read_bytes() != (tmp_path / "a.fa").read_bytes()


def test_read_simulator_random_mode_and_errors(tmp_path):
    rc, out, _ = run("read_simulator", "-l", 33, "-n", 7, "-o", tmp_path / "r.fa")
    assert rc == 0 and out.startswith("no fasta file")
    recs = parse_sim(tmp_path / "r.fa")
    assert [h for h, _ in recs] == [f"simulated-{i}" for i in range(7)]
    assert all(len(s) == 33 and set(s) <= set("ACGT") for _, s in recs)
    assert run("read_simulator", "-n", 3)[0] == 1  # -o is required
    # more substitutions than positions: the reference's transcript error
    rc, _, err = run("read_simulator", "-i", os.path.join(GOLD, "ref_b.fa"), "-l", 4,
                     "--substitution_errors", 5, "-o", tmp_path / "x.fa")
    assert rc == 1 and "no more matches" in err


@pytest.mark.gpu
def test_cli_simulated_reads_are_found(tmp_path, gpu_device):
    """read_simulator -> search: every read's simulated origin is among its hits."""
    ref = os.path.join(GOLD, "ref_b.fa")  # ACGT only: the simulator's reference equals the index's
    rc, _, err = run("read_simulator", "-i", ref, "-l", 50, "-n", 200, "-e", 2, "-o", tmp_path / "r.fa")
    assert rc == 0, err
    out = tmp_path / "h.txt"
    rc, _, err = run("search", "-q", tmp_path / "r.fa", "-i", os.path.join(GOLD, IDX["b"]), "-e", 2, "-o", out)
    assert rc == 0, err
    hits = read_hits(out, 3)
    found = {(int(q), int(s), int(p)) for q, s, p in hits.tolist()}
    import re
    for i, (head, _) in enumerate(parse_sim(tmp_path / "r.fa")):
        m = re.search(r"seqid:(\d+), pos:(\d+), trans:([MSID]+)", head)
        seqid, pos, trans = int(m.group(1)), int(m.group(2)), m.group(3)
        lead_d = len(trans) - len(trans.lstrip("D"))  # leading deletions shift the start (policy P0)
        lead_i = len(trans) - len(trans.lstrip("I"))
        starts = {pos + k for k in range(0, lead_d + 1)} | {pos}
        assert any((2 * i, seqid, p) in found for p in starts) or lead_i > 0, (i, head)


@pytest.mark.gpu
def test_cli_dynamic_generator(tmp_path, gpu_device):
    """--dynamic_generator prints the partition and finds the golden hit set."""
    out = tmp_path / "h.txt"
    rc, so, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                      "-e", 2, "--dynamic_generator", "--emit-errors", "-o", out)
    assert rc == 0, err
    assert "  dynamic expansion:   true" in so
    part = [l for l in so.splitlines() if l.startswith("partition: [")]
    assert len(part) == 1 and sum(map(int, part[0][12:-1].split(","))) == 40
    from helpers import pset
    assert pset(hits_as_rows(read_hits(out, 4))) == pset(expected("a_lev_k2"))


@pytest.mark.gpu
@pytest.mark.parametrize("gen,k", [("backtracking", 2), ("h2-k2", 2), ("pigeon", 1)])
def test_cli_hamming_node_counts_before_limit(gen, k, tmp_path, gpu_device):
    """-d ham: search.cpp:207-208 print nodeCount<false> / weightedNodeCount<false>
    of the expanded scheme, and only then (search.cpp:226) limitToHamming it
    for the search; the hits are the limited scheme's."""
    import sahara_amd as sa
    from test_golden import read_fasta, SIGMA
    reads = read_fasta(os.path.join(GOLD, "reads_a.fa"), SIGMA["a"])
    m = len(reads[0])
    n = sa.BiFMIndex.load(os.path.join(GOLD, IDX["a"]), device=gpu_device).info()["n"]
    full = sa.search_scheme(gen, 0, k, m, hamming=False)
    limited = sa.search_scheme(gen, 0, k, m, hamming=True)
    nc, wnc = sa.scheme_counts(full, False, 6, n)
    lnc, lwnc = sa.scheme_counts(limited, False, 6, n)
    out = tmp_path / "h.txt"
    rc, so, err = run("search", "-q", os.path.join(GOLD, "reads_a.fa"), "-i", os.path.join(GOLD, IDX["a"]),
                      "-e", k, "-g", gen, "-d", "ham", "-o", out)
    assert rc == 0, err
    lines = so.splitlines()
    got_nc = float(next(ln for ln in lines if ln.startswith("node count: ")).split(": ")[1])
    got_wnc = float(next(ln for ln in lines if ln.startswith("weighted node count: ")).split(": ")[1])
    assert got_nc == nc and got_wnc == wnc
    # (this build's count DP visits only reachable (pos, e) states, which the
    # Hamming limit never removes: the limited scheme counts the same here;
    # upstream's nodeCount over the raw bounds may not, hence the order)
    assert (lnc, lwnc) == (nc, wnc)
