import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")


@pytest.fixture(scope="session")
def sw():
    import _swpkg
    return _swpkg.load()


@pytest.fixture(scope="session")
def oracle():
    import sw_oracle
    sw_oracle.lib()
    return sw_oracle


@pytest.fixture(scope="session")
def handle(sw):
    # the library's own kernel choices, whatever SW_* variables are set
    h = sw.Handle(0, env_opts=False)
    yield h
    h.close()


@pytest.fixture
def knobs(handle):
    """knobs(field=value, ...): sw_opts overrides on the session handle for
    one test (include/sw_amd.h field names; a string value is converted,
    "" = the library's choice), restored afterwards."""
    saved = handle.get_opts()

    def set_(**kw):
        conv = {}
        for k, v in kw.items():
            if isinstance(v, str) and k not in ("inter_variant", "trace_file"):
                v = int(v) if v.strip() else -1
            conv[k] = v
        handle.set_opts(**conv)
    yield set_
    handle.set_opts(saved)


def read_query(name):
    with open(os.path.join(GOLDEN, "queries", name + ".fasta")) as f:
        return "".join(f.read().split("\n")[1:])


def read_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return [int(x) for x in f.read().split()]


def path_score(q, s, mat, go, ge, al):
    """Score of an alignment's path (ops from (q_begin, s_begin)) under a gap
    of go for its first residue and ge for each further one: equal to the
    reported score whatever the tie rules, so it checks a traceback without
    trusting them."""
    i, j, sc, prev = al["q_begin"] - 1, al["s_begin"] - 1, 0, None
    for op in al["ops"]:
        if op == "M":
            sc += int(mat[q[i]][s[j]])
            i += 1
            j += 1
        else:
            sc -= ge if prev == op else go
            if op == "I":
                i += 1
            else:
                j += 1
        prev = op
    assert (i, j) == (al["q_end"], al["s_end"]), "the path ends at the end cell"
    return sc
