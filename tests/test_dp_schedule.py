"""DP step schedule on CPU (no GPU): the bucket launch splice and the stream program the
HIP executor captures into ONE graph per step (VERDICT r1 "fake-comm unit
test on the captured launch list").  Launches are fakes that record what ran where."""
import pytest

from cori_intml_examples_amd.models.executor_hip import (check_bucket_cover, splice_bucket_launches,
                                                          stream_program)
from cori_intml_examples_amd.parallel.dist import merge_buckets

# RPV DP step, backward order: head, dense, conv3, conv2, conv1 (flat ranges of the store)
GROUPS = [(547712, 547841), (23584, 547712), (5088, 23584), (448, 5088), (0, 448)]


def _fake_step(comm=True, optim_on_comm=True, bucket_bytes=1 << 20):
    base = [("prologue", None, "main"), ("conv_stack_fwd", None, "main"), ("dense_fwd0", None, "main"),
            ("dense_epi0", None, "main"), ("head", None, "main")]
    red_ready = [len(base)]                       # head slabs final after the head launch
    base.append(("dense_bwd0", None, "main"))
    red_ready.append(len(base))
    for i in (2, 1):
        base.append(("wgrad_dgrad_conv%d" % i, None, "main"))
        red_ready.append(len(base))
    base.append(("wgrad_conv0", None, "side"))
    red_ready.append(len(base))
    bucket_groups, spans = merge_buckets(GROUPS, bucket_bytes)
    inserts = [(max(red_ready[i] for i in bg), k) for k, bg in enumerate(bucket_groups)]
    fake = lambda k: (lambda s: None)      # noqa: E731
    per = [("reduce_b%d", fake, "side")]
    if comm:
        per.append(("allreduce_b%d", fake, "comm"))
        if optim_on_comm:
            per.append(("optim_b%d", fake, "comm"))
    launches, ready = splice_bucket_launches(base, inserts, per)
    return launches, ready, spans


def _run(launches):
    """Execute the stream program on fake streams: each stream is a list of launch names;
    a wait records (dst waits for src's last launch so far)."""
    tags = [l[2] for l in launches]
    ops = stream_program(tags)
    streams = {"main": [], "comm": []}
    deps = []        # (stream, position in that stream, (src stream, number of src launches seen))
    for op in ops:
        if op[0] == "wait":
            deps.append((op[1], len(streams[op[1]]), op[2], len(streams[op[2]])))
        else:
            streams[op[1]].append(launches[op[2]][0])
    return ops, streams, deps


def _happens_before(streams, deps, a, b):
    """True if launch a is ordered before launch b by stream order + waits (transitively)."""
    where = {n: (s, i) for s, names in streams.items() for i, n in enumerate(names)}
    target, start = where[a], where[b]

    def preds(node):
        s, i = node
        if i > 0:
            yield (s, i - 1)
        for dst, pos, src, cnt in deps:
            if dst == s and pos <= i and cnt > 0:
                yield (src, cnt - 1)

    stack, seen = list(preds(start)), set()
    while stack:
        node = stack.pop()
        if node == target:
            return True
        if node not in seen:
            seen.add(node)
            stack.extend(preds(node))
    return False


def test_dp_step_schedule_orders_reduce_allreduce_optim():
    launches, ready, spans = _fake_step()
    names = [l[0] for l in launches]
    assert len(spans) == 2 and ready == [names.index("optim_b0") + 1, names.index("optim_b1") + 1]
    ops, streams, deps = _run(launches)
    # comm stream carries exactly the all-reduces and the per-bucket updates, in bucket order
    assert streams["comm"] == ["allreduce_b0", "optim_b0", "allreduce_b1", "optim_b1"]
    for k in range(2):
        assert _happens_before(streams, deps, "reduce_b%d" % k, "allreduce_b%d" % k)
        assert _happens_before(streams, deps, "allreduce_b%d" % k, "optim_b%d" % k)
    # the dense bucket's all-reduce is forked BEFORE the conv backward and not ordered after it
    assert not _happens_before(streams, deps, "wgrad_dgrad_conv2", "allreduce_b0")
    assert names.index("allreduce_b0") < names.index("wgrad_dgrad_conv2")
    # the conv bucket's slab reduction sees every conv weight gradient
    for w in ("wgrad_dgrad_conv2", "wgrad_dgrad_conv1", "wgrad_conv0"):
        assert _happens_before(streams, deps, w, "reduce_b1")
    # the step ends with main joined to comm (the next step's prologue re-packs the updated
    # weights, so it must follow every optimizer launch)
    assert ops[-1] == ("wait", "main", "comm") or ("wait", "main", "comm") in ops[-3:]
    last_join = max(i for i, op in enumerate(ops) if op == ("wait", "main", "comm"))
    assert all(op[0] == "wait" for op in ops[last_join:])


def test_single_gpu_schedule_has_no_comm():
    launches, ready, spans = _fake_step(comm=False, bucket_bytes=1 << 62)
    ops, streams, _ = _run(launches)
    assert streams["comm"] == [] and len(spans) == 1
    assert streams["main"][-1] == "reduce_b0"


def test_segmented_split_points():
    """Without capture (torch.distributed data plane) the step is cut at bucket_ready."""
    launches, ready, _ = _fake_step(comm=False)
    names = [l[0] for l in launches]
    assert names[ready[0] - 1] == "reduce_b0" and names[ready[1] - 1] == "reduce_b1"


def test_bucket_cover():
    _, spans = merge_buckets(GROUPS, 1 << 20)
    check_bucket_cover(spans, 547841)
    with pytest.raises(AssertionError):
        check_bucket_cover(spans[:1], 547841)
    with pytest.raises(AssertionError):
        check_bucket_cover([(0, 10), (11, 20)], 20)
    with pytest.raises(AssertionError):
        check_bucket_cover([(0, 12), (10, 20)], 20)
    # any bucket size: spans tile the buffer in backward order
    for bb in (1, 512, 4096, 1 << 16, 1 << 30):
        bg, sp = merge_buckets(GROUPS, bb)
        check_bucket_cover(sp, 547841)
        assert [s[0] for s in sp] == sorted((s[0] for s in sp), reverse=True)


def test_linear_schedule_keeps_comm_on_main():
    launches, _, _ = _fake_step()
    tags = [l[2] for l in launches]
    ops = stream_program(tags, comm=False)
    assert all(op[0] == "run" and op[1] == "main" for op in ops)
    assert [launches[op[2]][0] for op in ops] == [l[0] for l in launches]


def test_splice_skips_buckets_a_factory_declines():
    """Hybrid plane: the xGMI bucket gets the fused kernel on main, the others RCCL + optimizer
    on the comm stream (a factory returning None skips that bucket)."""
    base = [("a", None, "main"), ("b", None, "main"), ("c", None, "main")]
    xk = 1
    per = [("reduce_b%d", lambda k: (lambda s: None), "side"),
           ("allreduce_b%d", lambda k: None if k == xk else (lambda s: None), "comm"),
           ("optim_b%d", lambda k: None if k == xk else (lambda s: None), "comm"),
           ("xgmi_b%d", lambda k: (lambda s: None) if k == xk else None, "main")]
    out, ready = splice_bucket_launches(base, [(1, 0), (3, 1)], per)
    names = [o[0] for o in out]
    assert names == ["a", "reduce_b0", "allreduce_b0", "optim_b0", "b", "c", "reduce_b1", "xgmi_b1"]
    assert ready == [4, 8]
    ops = stream_program([o[2] for o in out])
    comm = [out[op[2]][0] for op in ops if op[0] == "run" and op[1] == "comm"]
    assert comm == ["allreduce_b0", "optim_b0"] and ops[-1] == ("wait", "main", "comm")


def test_comm_optimizer_waits_for_later_pack_readers():
    """a comm-stream optimizer writes its layers' bf16 packs, so it must be
    ordered after every later main-stream launch that reads one of them.  Legacy-shaped step
    (wide convs: separate dgrad launches after each wgrad), 1 MiB buckets: bucket 1 holds
    conv3's weights, whose pack dgrad_conv3 reads after the bucket's slabs are final."""
    from cori_intml_examples_amd.models.executor_hip import defer_after_readers
    fake = lambda k: (lambda s: None)      # noqa: E731
    base = [("conv_fwd%d" % i, None, "main") for i in range(4)] + [("head", None, "main"),
                                                                    ("dense_bwd0", None, "main")]
    red_ready = [5, 6]
    for i in (3, 2, 1, 0):
        base.append(("wgrad_conv%d" % i, None, "side"))
        red_ready.append(len(base))
        if i:
            base.append(("dgrad_conv%d" % i, None, "main"))
    spans = [(30_000_000, 34_515_201), (20_000_000, 30_000_000), (1_000, 20_000_000), (0, 1_000)]
    inserts = [(red_ready[0], 0), (red_ready[2], 1), (red_ready[3], 2), (red_ready[5], 3)]
    per = [("reduce_b%d", fake, "side"), ("allreduce_b%d", fake, "comm"), ("optim_b%d", fake, "comm")]
    launches, _ = splice_bucket_launches(base, inserts, per)
    readers = [("dense_bwd0", 30_000_000, 34_515_000), ("dgrad_conv3", 20_000_000, 30_000_000),
               ("dgrad_conv2", 1_000, 10_000_000), ("dgrad_conv1", 10_000_000, 20_000_000)]
    before = [l[0] for l in launches]
    assert before.index("optim_b1") < before.index("dgrad_conv3")        # the race ADVICE found
    out = defer_after_readers(launches, "optim_b%d", spans, readers)
    names = [l[0] for l in out]
    assert sorted(names) == sorted(before)
    ops, streams, deps = _run(out)
    for rn, rlo, rhi in readers:
        for k, (lo, hi) in enumerate(spans):
            if rlo < hi and rhi > lo:
                assert _happens_before(streams, deps, rn, "optim_b%d" % k), (rn, k, names)
    # the all-reduces did not move: bucket 1's still overlaps conv3's dgrad
    assert names.index("allreduce_b1") < names.index("dgrad_conv3")
    for k in range(4):
        assert _happens_before(streams, deps, "allreduce_b%d" % k, "optim_b%d" % k)
    # nothing to defer: the RPV step's order is unchanged
    rpv, _, sp = _fake_step()
    assert defer_after_readers(rpv, "optim_b%d", sp, [("dense_bwd0", 23584, 547712)]) == rpv
