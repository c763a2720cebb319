"""Tracing / engine counters."""
import euler_amd as ea
from euler_amd.utils import trace


def test_stage_timer_and_engine_stats():
    ea.synthetic_graph(500, 4, 32, feature_dim=4)
    trace.reset_engine_stats()
    t = trace.StageTimer()
    for _ in range(3):
        with trace.trace_range("neighbors", timer=t):
            ea.get_full_neighbor([1, 2, 3], ["0"])
    s = t.summary()
    assert s["neighbors"]["count"] == 3 and s["neighbors"]["total_ms"] >= 0
    assert "neighbors" in t.report()
    st = trace.engine_stats()
    assert st["queries"] == 3 and st["dag_nodes"] >= 3 and st["compile_us"] >= 0
