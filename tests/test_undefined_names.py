"""CPU: no Python file of the repo reads a global name that is never bound
(tools/undef_check.py, symtable-based).  bench.py's GPU legs, the probes and
the tools run only on the GPU box; a NameError there would otherwise surface
only in the driver's run."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_undefined_globals():
    files = subprocess.run(["git", "ls-files", "*.py"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.split()
    assert "bench.py" in files
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "undef_check.py"), *files],
                       cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout


def test_checker_flags_an_undefined_name(tmp_path):
    p = tmp_path / "m.py"
    p.write_text("import os\ndef f():\n    return os.sep + not_bound_anywhere\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "undef_check.py"), str(p)],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "not_bound_anywhere" in r.stdout
