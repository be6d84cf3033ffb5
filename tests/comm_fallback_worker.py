"""CPU worker for tests/test_dp.py::test_rccl_failure_falls_back_collectively: RCCL data-plane
bring-up is made to fail in one phase, on ALL ranks or on ONE rank only, and dist.init must
vote the whole job onto the RCCL-free plane -- no rank raises, no rank hangs:

  all_init  every rank's communicator construction raises (a node whose RCCL cannot come up)
  one_init  only rank 1's construction raises (its peers' constructions succeed)
  uid       rank 0 cannot create the unique id (the others learn it from rank 0's broadcast)
  hang      rank 1's construction never returns (INTML_RCCL_INIT_TIMEOUT bounds the wait)
  late      rank 1's construction returns AFTER the deadline: the reaper aborts + closes it
  selftest  rank 1's numeric self-test fails (wrong sum in the captured all-reduce)
  ok        everything succeeds: the job keeps its communicator
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cori_intml_examples_amd.parallel import comm as C  # noqa: E402
from cori_intml_examples_amd.parallel import dist  # noqa: E402

SCENARIO = sys.argv[2] if len(sys.argv) > 2 else "all_init"
RANK = int(os.environ.get("RANK", "0"))


class _FakeModule:
    @staticmethod
    def unique_id():
        if SCENARIO == "uid":
            raise RuntimeError("ncclGetUniqueId: unhandled system error (injected)")
        return b"\0" * 128


class _FakeComm:
    aborted = []
    closed = 0

    def __init__(self, rank, size, device, timeout_s, uid=None):
        if SCENARIO == "all_init" or (SCENARIO == "one_init" and rank == 1):
            raise RuntimeError("ncclCommInitRank: unhandled system error (injected)")
        if SCENARIO == "hang" and rank == 1:
            time.sleep(3600)
        if SCENARIO == "late" and rank == 1:
            time.sleep(float(os.environ.get("INTML_RCCL_INIT_TIMEOUT", 4)) + 2.0)
        self.rank, self.size = rank, size

    def self_test(self, timeout_s=60.0):
        if SCENARIO == "selftest" and self.rank == 1:
            return "captured all-reduce wrong: max |err| 2 (injected)"
        return None

    def abort(self, why="aborted"):
        _FakeComm.aborted.append(why)

    def close(self):
        _FakeComm.closed += 1


def main(outdir):
    C.comm_mode = lambda *a, **k: "native"      # what a multi-GPU node selects
    C.NativeComm = _FakeComm
    C._module = lambda: _FakeModule
    t0 = time.time()
    st = dist.init()
    rep = {"rank": st.rank, "size": st.size, "xgmi_only": bool(st.xgmi_only), "comm": st.comm is not None,
           "plane": st.plane, "aborted": len(_FakeComm.aborted), "init_s": time.time() - t0}
    if SCENARIO == "late":
        # the late communicator must be aborted + closed by the reaper once it comes up
        deadline = time.time() + 20
        while time.time() < deadline and any(r["state"] == "pending" for r in C.abandoned_inits):
            time.sleep(0.1)
        rep["abandoned"] = [r["state"] for r in C.abandoned_inits]
        rep["aborted"], rep["closed"] = len(_FakeComm.aborted), _FakeComm.closed
    with open(os.path.join(outdir, "fb%d.json" % st.rank), "w") as f:
        json.dump(rep, f)
    if st.comm is not None:
        st.comm = None
    dist.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
    # (a thread abandoned inside a hung "RCCL init" must not keep the process alive)
    sys.stdout.flush()
    os._exit(0)
