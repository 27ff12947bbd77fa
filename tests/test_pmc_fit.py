"""CPU: tools/pmc_fit.py refuses rocprofv3 --pmc counter sets that do not fit
one pass (an over-full TCC set hangs rocprofv3 at start)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_fit  # noqa: E402


def test_committed_passes_fit():
    sets = [["FETCH_SIZE"], ["WRITE_SIZE"],
            "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum "
            "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE".split(),
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE".split()]
    for s in sets:
        assert pmc_fit.problems(s) == [], s


def test_overfull_sets_are_refused():
    # five distinct TCC counters (the shape of round 3's hung per-channel pass)
    tcc5 = "TCC_REQ TCC_TAG_STALL TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL TCC_HIT GRBM_GUI_ACTIVE".split()
    assert any(p.startswith("TCC: 5") for p in pmc_fit.problems(tcc5))
    assert pmc_fit.problems(["FETCH_SIZE", "WRITE_SIZE"])  # 3 + 2 TCC slots
    assert pmc_fit.problems(["FETCH_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"])
    assert pmc_fit.problems(["TA_BUSY_avr", "TA_FLAT_READ_WAVEFRONTS_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"])
    assert pmc_fit.problems(["XYZ_COUNT"])  # unknown block: refused, not guessed


def test_reductions_and_instances_count_once():
    assert pmc_fit.slots(["TCC_REQ_sum", "TCC_REQ", "TCC_REQ[3]", "TCC_REQ_max"]) == {"TCC": 1}


def test_cli_exit_codes():
    tool = os.path.join(ROOT, "tools", "pmc_fit.py")
    ok = subprocess.run([sys.executable, tool, "FETCH_SIZE"], capture_output=True, text=True)
    assert ok.returncode == 0
    bad = subprocess.run([sys.executable, tool, "FETCH_SIZE WRITE_SIZE"], capture_output=True,
                         text=True)
    assert bad.returncode == 1 and "does not fit" in bad.stderr
