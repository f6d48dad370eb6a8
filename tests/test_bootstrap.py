"""CPU: the drivers' RCCL-id bootstrap (driver_common.cpp share_comm_id),
which replaces HPX's locality bootstrap for bin/2d_nonlocal_distributed:
rank 0 serves the id on MASTER_ADDR:MASTER_PORT+1, the other ranks fetch it,
once per batch row.  Runs the harness tools/comm_id_check.cpp (bin/
comm_id_check, built with the drivers) with a stand-in id, no GPU."""
import os
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_comm_id_bootstrap_successive_rows(nranks):
    """The drivers' TCP bootstrap of the RCCL unique id (driver_common.cpp
    share_comm_id; rank 0 serves, the others fetch from MASTER_ADDR:
    MASTER_PORT+1) over several successive batch rows, with a stand-in id per
    row (no GPU): every rank receives rank 0's id of that row."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    exe = os.path.join(ROOT, "bin", "comm_id_check")
    rounds = 4
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port - 1))
        procs.append(subprocess.Popen([exe, str(rounds), "7"], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e
        outs.append(o.split("\n"))
    ids = [[l.split()[2] for l in o if l.startswith("round ")] for o in outs]
    assert all(len(i) == rounds for i in ids)
    for r in range(1, nranks):
        assert ids[r] == ids[0]
    assert len(set(ids[0])) == rounds  # a fresh id per row
