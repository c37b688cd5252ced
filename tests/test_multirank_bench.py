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
    got = [r for r in multirank_result if r["ranks"] == ranks]
    assert got, multirank_result
    r = got[0]
    assert r["rc"] == 0, r.get("stderr")
    line = r["line"]
    assert line["n_gpus"] == ranks and line["verified"] is True, line
    assert "gloo" in line["config"]["gather"]
