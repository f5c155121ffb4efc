"""The multi-rank gather protocol on the CPU:
tests/comm_protocol/fake_comm.cpp runs raytracing2-fork_amd/csrc/device/
rt2_comm_protocol.h — the same control flow rt2_comm.hip runs under RCCL —
with 2 and 3 ranks as threads over a fake transport whose collectives are
rendezvous with a deadline (the RCCL transport's watchdog).  Every failure site
(gather.prepare, gather.issue, check, render, agree.copy), on the first and the
last rank: every rank returns < 0 within the deadline; failures the agreement
sees make every rank return at once and issue no gather.  A mutant that
returns before the agreement (round 2's hang) must be caught."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "comm_protocol", "fake_comm.cpp")
INC = os.path.join(ROOT, "raytracing2-fork_amd", "csrc", "device")


def build_and_run(tmp_path, *defines):
    exe = str(tmp_path / ("fake_comm" + "".join(d.lower() for d in defines)))
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-Wall", "-Wextra", "-Werror", f"-I{INC}",
                    *[f"-D{d}" for d in defines], SRC, "-o", exe], check=True)
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    return p.returncode, [json.loads(line) for line in p.stdout.splitlines() if line.strip()]


def test_every_failure_site_fails_every_rank_without_hang(tmp_path):
    rc, cases = build_and_run(tmp_path)
    assert cases and rc == 0, [c for c in cases if not c["pass"]]
    sites = {(c["proto"], c["site"]) for c in cases}
    assert {("gather_slabs", "gather.prepare"), ("gather_slabs", "agree.copy"),
            ("render_host_gather", "check"), ("render_host_gather", "render"),
            ("render_host_gather", "agree.copy"), ("render_host_gather", "gather.issue")} <= sites
    for c in cases:
        if c["site"]:
            assert all(r < 0 for r in c["rc"]), c
        else:
            assert c["rc"] == [0] * c["n"] and c["gathers"] == c["n"], c


def test_harness_catches_an_early_return(tmp_path):
    rc, cases = build_and_run(tmp_path, "MUTANT_EARLY_RETURN")
    assert rc != 0
    bad = [c for c in cases if not c["pass"]]
    assert bad and all(c["site"] == "gather.prepare" for c in bad), bad


if __name__ == "__main__":
    pytest.main([__file__, "-v"])
