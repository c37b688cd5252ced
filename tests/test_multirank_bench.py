"""bench.py's multi-rank path (one process per rank, interleaved 8-row bands,
two-slot asynchronous gather to rank 0, rt_assemble_bands) run for real as
child processes: 2 and 3 ranks on the one GPU of the box, gloo in place of
RCCL (RCCL refuses two ranks on one device).  Every rank traces through the
C-ABI; rank 0 re-renders the whole frame alone and the gathered frame must be
bit-identical (--verify).  Started by tests/conftest.py before this process
touches the GPU; see scripts/multirank_check.py."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ranks", [2, 3])
def test_bench_multirank_gathered_frame_is_bit_identical(multirank_result, ranks):
    got = [r for r in multirank_result if r.get("ranks") == ranks and r.get("launcher") != "none"]
    assert got, multirank_result
    r = got[0]
    assert r["rc"] == 0, r.get("stderr")
    line = r["line"]
    assert line["n_gpus"] == ranks and line["verified"] is True, line
    assert "gloo" in line["config"]["gather"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("ranks", [3, 8])
def test_bench_single_process_multi_device_is_bit_identical(multirank_result, ranks):
    """bench.py --gpus N with no launcher drives rt_multi in one process; on this
    box the N devices are all cuda:0 (BENCH_SHARE_GPU=1 -> peer copies).  --gpus 8 runs the full C2 frame."""
    got = [r for r in multirank_result if r.get("ranks") == ranks and r.get("launcher") == "none"]
    assert got, multirank_result
    r = got[0]
    assert r["rc"] == 0, r.get("stderr")
    line = r["line"]
    assert line["n_gpus"] == ranks and line["verified"] is True, line
    assert line["config"]["launcher"].startswith("single process"), line["config"]
    assert "hipMemcpyPeerAsync" in line["config"]["gather"], line["config"]
    assert len(line["per_device_trace_ms"]) == ranks
    assert line["one_gpu"]["ms_per_frame"] > 0
    if ranks == 8:
        assert line["config"]["rays_per_step"] == 719275410  # the C2 golden's count
