"""bench.py's host-side logic that runs without a GPU: the measured exchange choice of the
multi-GPU line (every rank must pick the same exchange; warm-up must not decide)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_exchange_trial_alternates_and_keeps_the_faster_round():
    bench = _bench()
    calls, order = [], []
    # the first timed round of whichever exchange runs first carries a warm-up penalty
    cost = {"allreduce": 0.849, "sh": 0.859}
    seen = set()

    def timed(fn, k):
        kind = fn.kind
        order.append(kind)
        first = not seen
        seen.add(kind)
        return k * (cost[kind] + (0.1 if first else 0.0))

    def step_of(kind):
        def fn():
            calls.append(kind)
        fn.kind = kind
        return fn

    drains = []
    chosen, trial = bench.exchange_trial({"allreduce": step_of("allreduce"), "sh": step_of("sh")}, timed,
                                         lambda: drains.append(1))
    assert chosen == "allreduce"  # the fixed-order single round would have picked sh (0.949 > 0.859)
    assert order == ["allreduce", "sh", "allreduce", "sh"]
    assert abs(trial["allreduce"] - 0.849) < 1e-12 and abs(trial["sh"] - 0.859) < 1e-12
    assert calls == ["allreduce"] * 3 + ["sh"] * 3 and drains == [1]
