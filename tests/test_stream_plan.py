"""The batch call's stream plan and the HIP-graph capture rules (CPU only:
dis_batch_stream_plan / dis_check_stream_plan need no device). The rules were
measured on HIP 7.2 with tools/capture_probe.hip and
tools/repro_sibling_capture.sh: a sub-batch stream left
unjoined makes hipStreamEndCapture fail, leaves the stream in capture mode and
writes a handle that is not a graph; a wait on an event recorded before the
capture is silently dropped from the graph; a sibling edge between sub-batch
streams crashes hipStreamEndCapture on the product's graph (the r05 crash)."""
import pytest

REC, WAIT, WORK = 0, 1, 2


@pytest.fixture(scope="module")
def d(disflow_mod):
    return disflow_mod


@pytest.mark.parametrize("nsub", range(2, 9))
def test_product_plans_keep_the_capture_rules(d, nsub):
    nstages = 9  # front end, levels 6..1, back end: 1080p MEDIUM
    ops = d.batch_stream_plan(nsub, nstages)
    assert d.check_stream_plan(ops, 1 + nsub, 1 + nsub) is None
    # shape: fork, every sub-batch's stages stage-major, joins
    assert ops[0] == (REC, 0, 0, -1)
    assert [o for o in ops if o[0] == WAIT and o[2] == 0] == [(WAIT, 1 + k, 0, -1) for k in range(nsub)]
    work = [o for o in ops if o[0] == WORK]
    assert work == [(WORK, 1 + k, -1, t) for t in range(nstages) for k in range(nsub)]
    assert ops[-2:] == [(REC, nsub, nsub, -1), (WAIT, 0, nsub, -1)]


def _fork(n):
    return [(REC, 0, 0, -1)] + [(WAIT, 1 + k, 0, -1) for k in range(n)]


def test_unjoined_stream_is_refused(d):
    # probe mode 5: sub-batch stream 2 never joins back
    ops = _fork(2) + [(WORK, 1, -1, 0), (WORK, 2, -1, 0), (REC, 1, 1, -1), (WAIT, 0, 1, -1)]
    why = d.check_stream_plan(ops, 3, 3)
    assert why and "R4" in why and "stream 2" in why


def test_work_after_the_join_is_refused(d):
    ops = _fork(1) + [(WORK, 1, -1, 0), (REC, 1, 1, -1), (WAIT, 0, 1, -1), (WORK, 1, -1, 1)]
    assert "R4" in d.check_stream_plan(ops, 2, 2)


def test_sibling_edges_are_refused(d):
    # a barrier between the sub-batch streams in the middle of the call: HIP 7.2
    # crashes inside hipStreamEndCapture on the product's graph with it
    # (tools/repro_sibling_capture.sh; the r05 crash), so the checker refuses
    # any wait of a sub-batch stream on another sub-batch stream's event
    ops = _fork(2) + [(WORK, 1, -1, 0), (WORK, 2, -1, 0),
                      (REC, 1, 1, -1), (REC, 2, 2, -1), (WAIT, 1, 2, -1), (WAIT, 2, 1, -1),
                      (WORK, 1, -1, 1), (WORK, 2, -1, 1),
                      (REC, 1, 1, -1), (WAIT, 0, 1, -1), (REC, 2, 2, -1), (WAIT, 0, 2, -1)]
    why = d.check_stream_plan(ops, 3, 3)
    assert why and "R5" in why and "sibling" in why
    # a transitive join is one too
    ops = _fork(2) + [(WORK, 1, -1, 0), (WORK, 2, -1, 0), (REC, 2, 2, -1), (WAIT, 1, 2, -1),
                      (REC, 1, 1, -1), (WAIT, 0, 1, -1)]
    assert "R5" in d.check_stream_plan(ops, 3, 3)


def test_stale_event_is_refused(d):
    # probe mode 3: a wait on an event not recorded in this capture is silently
    # dropped from the graph by HIP -- the checker refuses it
    ops = [(WAIT, 1, 1, -1)] + _fork(1)
    assert "R2" in d.check_stream_plan(ops, 2, 2)


def test_work_outside_the_capture_is_refused(d):
    ops = [(REC, 0, 0, -1), (WORK, 2, -1, 0), (WAIT, 1, 0, -1), (REC, 1, 1, -1), (WAIT, 0, 1, -1)]
    assert "R3" in d.check_stream_plan(ops, 3, 2)


def test_plan_argument_checks(d):
    import ctypes
    L = d.lib()
    n = ctypes.c_int()
    assert L.dis_batch_stream_plan(1, 3, None, 0, ctypes.byref(n)) == d.DIS_ERR_INVALID_ARGUMENT
    assert L.dis_batch_stream_plan(9, 3, None, 0, ctypes.byref(n)) == d.DIS_ERR_INVALID_ARGUMENT
    assert L.dis_batch_stream_plan(2, 3, None, 0, ctypes.byref(n)) == d.DIS_OK and n.value == 1 + 2 + 6 + 4
    small = (ctypes.c_int * 4)()
    assert L.dis_batch_stream_plan(2, 3, small, 1, ctypes.byref(n)) == d.DIS_ERR_INVALID_ARGUMENT
    assert "range" in d.check_stream_plan([(REC, 5, 0, -1)], 2, 1)
    assert "range" in d.check_stream_plan([(WAIT, 1, 7, -1)], 2, 1)
