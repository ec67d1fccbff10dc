"""Sanitizer builds of the host code (race detection / sanitizers): the multithreaded VCF
ingest (csrc/vcf_ingest.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer, and the C restatement of the oracle (oracle/sfs_oracle_c.c, OpenMP) under ASan +
UBSan.  Drivers in tests/sanitize/ are compiled with the sources here (g++ / gcc, host only: GPU
sanitizers are not available on the MI355X pool) and run on the golden VCFs and on larger
synthetic ones (many parse chunks, BGZF blocks, a late #CHROM line, error lines); every thread count
must give the same digest, no sanitizer may report, and the record counts must equal the normal
library's.  CPU only."""
import gzip
import os
import re
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")
SRC = os.path.join(REPO, "2dsfs-scan_amd", "csrc")
FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer"]
ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
           TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
           SFS2D_VCF_MERGE_CHUNK="61")   # the dict merge sharded over every thread even on small inputs

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")


def _build(out, cmd):
    r = subprocess.run(cmd + ["-o", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


@pytest.fixture(scope="module")
def drivers(tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    inc = ["-I", os.path.join(REPO, "include")]
    ingest = [os.path.join(SRC, "vcf_ingest.cpp"), os.path.join(HERE, "sanitize", "ingest_driver.cpp"), "-lz", "-pthread"]
    return {
        "ingest_asan": _build(str(d / "ingest_asan"), ["g++", "-std=c++17", *FLAGS, "-fsanitize=address,undefined",
                                                       "-fno-sanitize-recover=all", *inc, *ingest]),
        "ingest_tsan": _build(str(d / "ingest_tsan"), ["g++", "-std=c++17", *FLAGS, "-fsanitize=thread", *inc, *ingest]),
        "oracle_asan": _build(str(d / "oracle_asan"), ["gcc", "-std=c11", *FLAGS, "-fopenmp", "-fsanitize=address,undefined",
                                                       "-fno-sanitize-recover=all", os.path.join(REPO, "oracle", "sfs_oracle_c.c"),
                                                       os.path.join(HERE, "sanitize", "oracle_driver.c"), "-lm"]),
    }


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    sys.path.insert(0, HERE)
    sys.path.insert(0, GOLD)
    from gen_golden_vcf import bgzf_bytes
    from test_vcf_ingest import SAMPLES, synth_vcf, write_popmap
    d = tmp_path_factory.mktemp("vcf")
    pm = str(d / "pm.txt")
    write_popmap(pm, [(s, ["uv", "bv", "x"][i % 3]) for i, s in enumerate(SAMPLES) if i != 4])
    files = [(os.path.join(GOLD, "vcf_test.vcf.gz"), os.path.join(GOLD, "popmap_3pop.txt")),
             (os.path.join(GOLD, "vcf_test_plain.vcf.gz"), os.path.join(GOLD, "popmap_ref.txt"))]
    big = str(d / "big.vcf.gz")
    open(big, "wb").write(gzip.compress(synth_vcf(40000, SAMPLES, seed=5), 1))
    late = str(d / "late.vcf")
    open(late, "wb").write(synth_vcf(20000, SAMPLES, seed=6, late_header=True))
    blk = str(d / "blocks.vcf.gz")
    open(blk, "wb").write(bgzf_bytes(synth_vcf(30000, SAMPLES, seed=9).replace(b"\r\n", b"\n"), block=5000))
    bad = str(d / "bad.vcf.gz")
    open(bad, "wb").write(gzip.compress(synth_vcf(30000, SAMPLES, seed=2, bad=(25000, "chr1\t5\t.\tA\tC\t.\tPASS\tX")), 1))
    files += [(big, pm), (late, pm), (blk, pm), (bad, pm)]
    return files


def _run(exe, args, timeout=600):
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=ENV, timeout=timeout)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, \
        r.stderr[-4000:]
    return r.stdout


@pytest.mark.parametrize("kind,threads", [("ingest_asan", "1,3,16"), ("ingest_tsan", "2,8")])
def test_ingest_under_sanitizers(drivers, inputs, kind, threads):
    sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
    from sfs2d import vcf as V
    out = _run(drivers[kind], [threads] + [x for f in inputs for x in f])
    lines = out.strip().split("\n")
    assert len(lines) == len(inputs) * len(threads.split(","))
    by_file = {}
    for ln in lines:
        path = ln.split(" threads=")[0]
        by_file.setdefault(path, set()).add(re.sub(r" threads=\d+", "", ln))
    for (vcf, pm) in inputs:
        got = by_file[vcf]
        assert len(got) == 1, got                       # every thread count: the same result / error
        line = next(iter(got))
        if " rc=" in line:                             # the error input: an error, as the library raises
            with pytest.raises((IndexError, ValueError)):
                V.read_vcf(vcf, pm)
            continue
        n = int(re.search(r"records=(\d+)", line).group(1))
        assert n == V.read_vcf(vcf, pm).n


def test_oracle_c_under_sanitizers(drivers):
    out = _run(drivers["oracle_asan"], [])
    assert re.match(r"windows=\d+ digest=", out)
