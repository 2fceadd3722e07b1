"""Every reference citation (``gpmpc/<file>.py:N``, ``scripts/run_gp_mpc.py:N``, ...) in the
boundary header, the package, the oracle, the tests and the docs points at lines that exist in
/root/reference, and the key boundary citations point at the symbol they name.  Skipped when the
reference tree is absent (the GPU box)."""

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")
FILES = {"gp.py": "gpmpc/gp.py", "mpc.py": "gpmpc/mpc.py", "gpmpc.py": "gpmpc/gpmpc.py",
         "plotting.py": "gpmpc/plotting.py", "run_gp_mpc.py": "scripts/run_gp_mpc.py",
         "gp_mpc_config.yaml": "scripts/gp_mpc_config.yaml", "pyproject.toml": "pyproject.toml",
         "install_acados.sh": "install_acados.sh"}
PAT = re.compile(r"\b(gp|mpc|gpmpc|plotting|run_gp_mpc)\.py:(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)"
                 r"|\b(gp_mpc_config\.yaml|pyproject\.toml|install_acados\.sh):(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)")
SOURCES = ["include", "gp-mpc_amd", "oracle", "tests", "tools", "bench.py", "__graft_entry__.py", "DESIGN.md",
           "INTEGRATION.md", "README.md", "BASELINE.md"]

pytestmark = pytest.mark.skipif(not REF.is_dir(), reason="reference tree not present")


def _ref_lines(name):
    return (REF / FILES[name]).read_text().splitlines()


def _citations():
    for src in SOURCES:
        p = ROOT / src
        files = [p] if p.is_file() else [f for f in p.rglob("*") if f.is_file() and f.suffix in
                                         (".py", ".h", ".hip", ".cpp", ".md", ".sh", ".txt", "")]
        for f in files:
            if "lib" in f.parts or "build" in f.parts or f.name.startswith("."):
                continue
            try:
                text = f.read_text()
            except UnicodeDecodeError:
                continue
            for ln, line in enumerate(text.splitlines(), 1):
                for m in PAT.finditer(line):
                    name = (m.group(1) + ".py") if m.group(1) else m.group(3)
                    spec = m.group(2) or m.group(4)
                    for part in spec.split(","):
                        lo, _, hi = part.partition("-")
                        yield f"{f.relative_to(ROOT)}:{ln}", name, int(lo), int(hi or lo)


def test_every_citation_is_in_range():
    bad = []
    n = 0
    for where, name, lo, hi in _citations():
        n += 1
        nl = len(_ref_lines(name))
        if not (1 <= lo <= hi <= nl):
            bad.append(f"{where}: {name}:{lo}-{hi} (file has {nl} lines)")
    assert n > 100, n
    assert not bad, "\n".join(bad)


# (repo file, cited reference file, range, text that must occur in the cited lines)
KEY = [
    ("include/gpmpc_mi355x.h", "gpmpc.py", (334, 368), "def select_action"),
    ("include/gpmpc_mi355x.h", "mpc.py", (185, 185), "assert status in [0, 2]"),
    ("include/gpmpc_mi355x.h", "mpc.py", (58, 58), "AcadosOcpSolver"),
    ("include/gpmpc_mi355x.h", "mpc.py", (62, 62), "acados_solver.reset()"),
    ("include/gpmpc_mi355x.h", "gpmpc.py", (105, 107), "AcadosOcpSolver"),
    ("include/gpmpc_mi355x.h", "gpmpc.py", (309, 310), "uh_0 = -1e-8"),
    ("include/gpmpc_mi355x.h", "mpc.py", (157, 158), "uh_0 = tol"),
    ("include/gpmpc_mi355x.h", "gp.py", (72, 85), "def gpytorch_predict2casadi"),
    ("gp-mpc_amd/gpmpc/mpc.py", "mpc.py", (15, 15), "U_EQ"),
    ("gp-mpc_amd/gpmpc/mpc.py", "mpc.py", (42, 45), "Q = np.diag(q_mpc)"),
    ("gp-mpc_amd/gpmpc/mpc.py", "mpc.py", (172, 186), "def select_action"),
    ("gp-mpc_amd/gpmpc/mpc.py", "mpc.py", (188, 193), "def reference_trajectory"),
    ("gp-mpc_amd/gpmpc/mpc.py", "mpc.py", (60, 63), "def reset"),
    ("gp-mpc_amd/gpmpc/gpmpc.py", "gpmpc.py", (18, 18), "U_EQ"),
    ("gp-mpc_amd/gpmpc/gpmpc.py", "gpmpc.py", (97, 108), "AcadosOcpSolver"),
    ("gp-mpc_amd/gpmpc/gpmpc.py", "gpmpc.py", (113, 151), "def preprocess_data"),
    ("gp-mpc_amd/gpmpc/gpmpc.py", "gpmpc.py", (509, 514), "def reference_trajectory"),
    ("gp-mpc_amd/gpmpc/learning.py", "run_gp_mpc.py", (42, 72), "def run_evaluation"),
    ("gp-mpc_amd/gpmpc/learning.py", "run_gp_mpc.py", (75, 83), "def sample_data"),
    ("gp-mpc_amd/gpmpc/learning.py", "run_gp_mpc.py", (86, 137), "def learn"),
    ("gp-mpc_amd/gpmpc/plotting.py", "plotting.py", (158, 181), "def make_quad_plots"),
    ("gp-mpc_amd/gpmpc/plotting.py", "plotting.py", (184, 228), "def plot_quad_eval"),
    ("oracle/gpmpc_oracle.py", "mpc.py", (157, 162), "uh = tol"),
    ("oracle/gpmpc_oracle.py", "gpmpc.py", (425, 498), "def propagate_constraint_limits"),
]


@pytest.mark.parametrize("src,name,rng,text", KEY)
def test_key_citation_points_at_its_symbol(src, name, rng, text):
    cites = {(n, lo, hi) for where, n, lo, hi in _citations() if where.rsplit(":", 1)[0] == src}
    assert (name, *rng) in cites, f"{src} does not cite {name}:{rng[0]}-{rng[1]}"
    lines = _ref_lines(name)[rng[0] - 1:rng[1]]
    assert any(text in ln for ln in lines), f"{name}:{rng[0]}-{rng[1]} does not contain {text!r}"
