"""Task farm with CPU "fake GPU" engines (SURVEY.md §4.3 "Task-farm tests"): scheduling,
AsyncResult fields, stdout capture, publish_data streaming, cancellation (Stop /
Restart), engine crash -> task error, SPMD ``%%px``."""
import os
import sys
import time

import cloudpickle
import pytest

from cori_intml_examples_amd import farm
from cori_intml_examples_amd.farm import magics

# engines cannot import this test module: ship its functions by value (as notebook
# functions defined in __main__ are)
cloudpickle.register_pickle_by_value(sys.modules[__name__])


@pytest.fixture(scope="module")
def cluster():
    cid = "pytest_%d" % os.getpid()
    cl = farm.start_cluster(2, cluster_id=cid, cpu_only=True, abort_grace=1.0, timeout=120)
    c = cl.client()
    yield cl, c
    c.close()
    cl.stop()


def _square(x, hold=0.0):
    import time
    time.sleep(hold)          # long enough that one engine cannot drain the queue alone
    print("square of", x)
    return x * x


def _publisher(n):
    from cori_intml_examples_amd.farm import publish_data
    for i in range(n):
        publish_data({"status": "Ended Epoch", "epoch": i, "history": {"loss": list(range(i + 1))}})
        time.sleep(0.05)
    return "done"


def test_ids_and_load_balanced(cluster):
    _, c = cluster
    assert c.ids == [0, 1]
    lv = c.load_balanced_view()
    ars = [lv.apply(_square, i, 0.3) for i in range(8)]
    assert [a.get(30) for a in ars] == [i * i for i in range(8)]
    assert {a.engine_id for a in ars} == {0, 1}          # both engines got work
    a = ars[3]
    assert a.ready() and a.successful() and a.stdout == "square of 3\n" and a.stderr == ""
    assert a.started is not None and a.completed >= a.started
    assert (a.completed - a.started).total_seconds() >= 0       # DistHPO_rpv.ipynb:217 usage
    assert lv.map_sync(_square, [1, 2, 3]) == [1, 4, 9]


def test_load_balanced_over_target_list(cluster):
    """A view restricted to an explicit target list spreads its tasks over every listed
    engine (it once sent all of them to the first one, serialising a whole search)."""
    _, c = cluster
    lv = c.load_balanced_view(targets=[0, 1])
    ars = [lv.apply(_square, i, 0.2) for i in range(4)]
    assert [a.get(30) for a in ars] == [i * i for i in range(4)]
    assert sorted(a.engine_id for a in ars) == [0, 0, 1, 1]
    one = c.load_balanced_view(targets=[1])
    ars = [one.apply(_square, i) for i in range(3)]
    assert [a.get(30) for a in ars] == [0, 1, 4] and {a.engine_id for a in ars} == {1}


_SHIPPED_GLOBAL = {}


def _count_calls():
    # a by-value function's module globals are rebuilt per task; the engine namespace is not
    _SHIPPED_GLOBAL["n"] = _SHIPPED_GLOBAL.get("n", 0) + 1
    ns = farm.engine_namespace()
    ns["calls"] = ns.get("calls", 0) + 1
    return ns["calls"], _SHIPPED_GLOBAL["n"]


def test_engine_namespace_persists(cluster):
    _, c = cluster
    v = c[0]
    first = v.apply_sync(_count_calls)
    second = v.apply_sync(_count_calls)
    assert second[0] == first[0] + 1 and second[1] == 1
    assert v.pull("calls") == second[0]          # same dict as push/pull/%%px


def test_publish_data_streams(cluster):
    _, c = cluster
    a = c.load_balanced_view().apply(_publisher, 5)
    assert a.get(30) == "done"
    assert a.data["epoch"] == 4 and a.data["status"] == "Ended Epoch"
    assert a.data["history"]["loss"] == [0, 1, 2, 3, 4]


def test_direct_view_spmd(cluster):
    _, c = cluster
    dv = c[:]
    dv.execute("import os\nrank = int(os.environ['RANK'])\nhistory = type('H', (), {})()\n"
               "history.epoch = [rank, rank + 1]", block=True)
    assert dv.get("rank") == [0, 1]
    assert c[1].get("history.epoch") == [1, 2]           # expression pull, DistTrain_rpv.ipynb:310
    dv["w"] = 5
    assert dv.pull("w * rank") == [0, 5]
    dv.scatter("part", list(range(6)), block=True)
    assert sorted(dv.gather("part")) == list(range(6))
    ar = magics.px("print('engine', rank)", client=c, verbose=False)
    assert ar.stdout == ["engine 0\n", "engine 1\n"]
    # engine id == DP rank == GPU slot (the reference's ids and ranks differ)
    assert c[:].apply_sync(lambda: int(os.environ["WORLD_SIZE"])) == [2, 2]


def test_remote_error(cluster):
    _, c = cluster

    def boom():
        raise ValueError("bad hyper-parameter")

    with pytest.raises(farm.RemoteError) as ei:
        c[0].apply_sync(boom)
    assert ei.value.ename == "ValueError" and "bad hyper-parameter" in ei.value.evalue
    assert "Traceback" in ei.value.traceback


def _sleeper(n):
    for _ in range(n):
        time.sleep(0.05)
    return n


def _cooperative():
    from cori_intml_examples_amd.farm import should_stop
    i = 0
    while i < 400:
        try:
            time.sleep(0.05)
        except KeyboardInterrupt:
            pass
        if should_stop():
            return "stopped at %d" % i
        i += 1
    return "finished"


def _stubborn():
    while True:
        try:
            time.sleep(0.05)
        except KeyboardInterrupt:
            pass


def test_abort_queued_and_running(cluster):
    _, c = cluster
    lv = c.load_balanced_view()
    busy = [lv.apply(_sleeper, 40) for _ in range(2)]
    queued = lv.apply(_square, 7)
    time.sleep(0.3)
    queued.abort()
    with pytest.raises(farm.TaskAborted):
        queued.get(10)
    for b in busy:
        b.abort()
        with pytest.raises(farm.TaskAborted):
            b.get(10)
    # cooperative stop: the task sees should_stop() and returns normally
    coop = c[0].apply_async(_cooperative)
    time.sleep(0.5)
    coop.abort()
    assert coop.get(10).startswith("stopped")


def test_hard_kill_and_crash_restart(cluster):
    _, c = cluster
    st = c[1].apply_async(_stubborn)
    time.sleep(0.5)
    st.abort(grace=0.5)
    with pytest.raises(farm.TaskAborted):
        st.get(20)

    def crash():
        os._exit(3)

    cr = c[0].apply_async(crash)
    with pytest.raises(farm.EngineError):
        cr.get(20)
    # both engines come back and take work again
    deadline = time.time() + 60
    while time.time() < deadline and len(c.ids) < 2:
        time.sleep(0.2)
    assert c.ids == [0, 1]
    assert c[0].apply_sync(_square, 4) == 16 and c[1].apply_sync(_square, 5) == 25
    st = c.queue_status()
    assert st[0]["restarts"] >= 1 and st[1]["restarts"] >= 1


def test_ipcluster_arg_parsing():
    a = magics.parse_ipcluster_args("-N 1 -n 4 -m numpy json -J mycluster -t 10:00")
    assert a["num_engines"] == 4 and a["modules"] == ["numpy", "json"] and a["name"] == "mycluster"
    d = magics.parse_ipcluster_args("")
    assert d["name"] == "ipyparallel" and d["num_nodes"] == 1 and d["queue"] == "interactive"


def test_runtime_dir_rejects_foreign_permissions(tmp_path, monkeypatch):
    """A pre-created group/world-accessible runtime dir (another local user could plant a
    connection file there) and a world-readable connection file are refused."""
    from cori_intml_examples_amd.farm import protocol as P
    d = tmp_path / "farm"
    d.mkdir()
    os.chmod(d, 0o777)
    monkeypatch.setenv("INTML_FARM_DIR", str(d))
    with pytest.raises(P.InsecurePathError):
        P.runtime_dir()
    os.chmod(d, 0o700)
    assert P.runtime_dir() == str(d)
    link = tmp_path / "link"
    link.symlink_to(d)
    monkeypatch.setenv("INTML_FARM_DIR", str(link))
    with pytest.raises(P.InsecurePathError):
        P.runtime_dir()
    monkeypatch.setenv("INTML_FARM_DIR", str(d))
    path = P.write_connection_file(P.new_connection_info("sec"))
    assert P.read_connection_file("sec")["cluster_id"] == "sec"
    os.chmod(path, 0o644)
    with pytest.raises(P.InsecurePathError):
        P.read_connection_file("sec")


def test_resource_usage_telemetry(cluster):
    """Engines report their resources (host RSS; HBM and GPU id on GPU engines) and the
    controller serves them in queue_status / ModelController.get_resource_usage (the
    reference's stub, hpo_widgets.py:366-367)."""
    from cori_intml_examples_amd.widgets import ModelController
    cl, c = cluster
    mc = ModelController(client=c)
    deadline = time.time() + 10
    st = {}
    while time.time() < deadline:
        st = mc.get_resource_usage()
        if all("rss_bytes" in st.get(e, {}) for e in c.ids):
            break
        time.sleep(0.3)
    for e in c.ids:
        assert st[e]["rss_bytes"] > 10 << 20 and "gpu" in st[e] and "queue" in st[e], st
