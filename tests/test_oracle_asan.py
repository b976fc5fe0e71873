"""The oracle's CPU tests once more against its ASan/UBSan build (oracle/Makefile
`asan`): the golden, chain, layer-walk and field-getter oracle tests run in a child
pytest with libasan preloaded and RPKT_ORACLE_BUILD=asan, so any out-of-bounds read,
use-after-free or undefined behaviour in the C restatement fails this test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUITES = ["tests/test_oracle_golden.py", "tests/test_oracle_chain.py",
          "tests/test_oracle_layers.py", "tests/test_oracle_fields.py",
          "tests/test_oracle_batch.py", "tests/test_oracle_fuzz_layouts.py"]


@pytest.mark.slow
def test_oracle_suites_clean_under_asan_ubsan():
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                             text=True).stdout.strip()
    if not os.path.isabs(libasan):
        pytest.skip("gcc has no libasan here")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"])
    env = dict(os.environ)
    # libasan first; whatever the environment already preloads stays after it
    env["LD_PRELOAD"] = ":".join(x for x in (libasan, os.environ.get("LD_PRELOAD", "")) if x)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:exitcode=99"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1:exitcode=98"
    env["RPKT_ORACLE_BUILD"] = "asan"
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu",
                        "-p", "no:cacheprovider"] + SUITES, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
    assert " passed" in r.stdout, tail
