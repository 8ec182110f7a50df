"""the CPU restatement (oracle/oracle.cpp) and libecc's pure-host C++
(host/events_io.cpp, host/aeclustering.cpp) built with -fsanitize=address,undefined and driven
over every stage (oracle/sanitize_main.cpp: downsample, dedup, k-means incl. the ref-compat
loop, SAE/arc corners in both border modes, NMS, tracker, eps-lists, float-cloud DBSCAN and
radius, OPTICS, EVT 2.0/3.0 encode -> file -> probe -> read -> decode, reslicing, CSV, AEClustering
+ flow + writers) on empty, single-event, ragged and multi-slice streams.  Any report fails."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_restatement_and_host_code_are_sanitizer_clean(tmp_path):
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "sanitize"], check=True, capture_output=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1:detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(ROOT / "oracle" / "_asan" / "sanitize_main"), str(tmp_path)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.count(" ok") == 4
