"""The multi-GPU stripe planner (flearn_amd.dist.StripeModel / plan_stripes): the two-stage
pipeline model behind bench.py's stripe choice, and the plans it produces."""
import pytest

from flearn_amd.dist import ALIGN, ShardPlan, StripeModel, plan_shards, plan_stripes, shard_candidates


def test_makespan_two_stage_pipeline():
    m = StripeModel(a_r=1.0, b_r=0.0, a_g=2.0, b_g=0.0)
    # reduces end at 1, 2, 3; gathers run back to back from t=1: 3, 5, 7
    assert m.makespan((64, 64, 64)) == (7.0, 3.0, 4.0)
    m = StripeModel(a_r=0.0, b_r=1.0, a_g=0.0, b_g=0.25)
    # reduce-bound: stripe 0's gather (48) hides behind stripe 1's reduce (64), only the last
    # stripe's gather (16) is exposed
    t, red, exp = m.makespan((192, 64))
    assert (t, red, exp) == (256 + 16, 256, 16)
    # gather-bound: stripe 1's gather waits for stripe 0's
    t, red, exp = StripeModel(0.0, 1.0, 0.0, 0.5).makespan((192, 64))
    assert (t, red, exp) == (192 + 96 + 32, 256, 64)


@pytest.mark.parametrize("cols", [1, 63, 64, 5001, 3_201_269, 10_820_957])
@pytest.mark.parametrize("model", [StripeModel.assumed(100, 8), StripeModel.assumed(1000, 8),
                                   StripeModel.assumed(100, 2), StripeModel(1e-6, 5e-9, 2e-6, 1e-8)])
def test_plan_covers_and_aligns(cols, model):
    w = plan_stripes(cols, model)
    assert all(x > 0 and x % ALIGN == 0 for x in w)
    assert sum(w) == -(-cols // ALIGN) * ALIGN
    assert 1 <= len(w) <= 8
    # never worse than the unstriped step
    assert model.makespan(w)[0] <= model.makespan((sum(w),))[0] + 1e-15


def test_plan_shapes_follow_the_bottleneck():
    lc = 3_201_269  # NS per rank at G = 8
    gather_bound = StripeModel(10e-6, 100 * 4 / 7e12, 30e-6, 7 * 4 / 150e9)
    w = plan_stripes(lc, gather_bound)
    assert len(w) >= 2 and w[0] < w[-1]  # start the gathers early
    reduce_bound = StripeModel(10e-6, 1000 * 4 / 7e12, 30e-6, 7 * 4 / 300e9)
    w = plan_stripes(lc, reduce_bound)
    assert len(w) >= 2 and w[0] > w[-1]  # hide all but a small last gather
    no_collective = StripeModel(10e-6, 100 * 4 / 7e12, 0.0, 0.0)
    assert len(plan_stripes(lc, no_collective)) == 1


def test_fit_recovers_lines():
    m = StripeModel.fit(8000, 1000, r_big=10 + 8000 * 2, r_small=10 + 1000 * 2, g_big=30 + 8000 * 5,
                        g_small=30 + 1000 * 5)
    assert m == pytest.approx(StripeModel(10, 2, 30, 5))
    m = StripeModel.fit(8000, 1000, 5.0, 6.0, 1.0, 1.0)  # noisy: slopes clamp at 0
    assert m.b_r == 0 and m.a_r == 6.0 and m.b_g == 0


def test_from_widths_layout():
    plan = ShardPlan.from_widths(1000, 4, 1, (64, 128, 64))
    assert plan.local_cols == 256 and plan.padded == 1024
    assert plan.global_begin(1) == 4 * 64 + 128  # stripe 1 starts at W*O_1, rank 1 after rank 0
    with pytest.raises(ValueError):
        ShardPlan.from_widths(1000, 4, 0, (64, 100))
    with pytest.raises(ValueError):
        ShardPlan.from_widths(10_000, 4, 0, (64, 64))


def test_makespan_with_replicated_tail():
    m = StripeModel(a_r=0.0, b_r=1.0, a_g=0.0, b_g=2.0)
    # stripe 0 reduced at 64, gathered 64..192; the tail's reduce (64..128) hides under it
    assert m.makespan((64,), rep=64) == (192.0, 128.0, 64.0)
    # a long tail: the step ends with the reduce, nothing exposed
    assert m.makespan((64,), rep=256) == (320.0, 320.0, 0.0)


@pytest.mark.parametrize("n_cols", [44_426, 11_699_112, 25_610_152])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_plan_shards_covers_exactly(n_cols, world):
    for model in (StripeModel.assumed(100, world), StripeModel.assumed(1000, world),
                  StripeModel(10e-6, 100 * 4 / 7e12, 0.0, 0.0)):
        widths, rep = plan_shards(n_cols, world, model)
        plan = ShardPlan.from_widths(n_cols, world, world - 1, widths, rep=rep)
        if rep:
            assert plan.full_cols == n_cols and world * sum(widths) + rep == n_cols
        else:
            assert plan.padded >= n_cols
        t = model.makespan(widths, rep)[0]
        w0 = plan_stripes(-(-n_cols // world), model)
        assert t <= model.makespan(w0)[0] + 1e-15  # never worse than the padded plan


def test_plan_shards_replicates_only_when_the_gather_dominates():
    p = 25_610_152  # NS
    # G = 2, one xGMI link: the gather of half the model takes longer than the reduce of it
    widths, rep = plan_shards(p, 2, StripeModel.assumed(100, 2))
    assert rep > 0.05 * p
    m = StripeModel.assumed(100, 2)
    assert m.makespan(widths, rep)[0] < 0.85 * m.makespan(plan_stripes(-(-p // 2), m))[0]
    # reduce-bound (1000 clients) or no collective: no replicated work beyond the alignment tail
    for m in (StripeModel.assumed(1000, 8), StripeModel(10e-6, 100 * 4 / 7e12, 0.0, 0.0)):
        assert plan_shards(11_699_112, 8, m)[1] < 8 * ALIGN


def test_replicated_tail_layout():
    plan = ShardPlan.from_widths(4 * 192 + 100, 4, 2, (128, 64), rep=100)
    assert plan.local_cols == 292 and plan.local_stripes == 192 and plan.full_cols == 868
    assert plan.segments() == [(0, 256, 128), (128, 4 * 128 + 128, 64), (192, 768, 100)]
    assert plan.local_to_global(191) == 4 * 128 + 128 + 63 and plan.local_to_global(192) == 768
    assert plan.local_to_global(291) == 867
    with pytest.raises(IndexError):
        plan.local_to_global(292)
    with pytest.raises(ValueError):  # the stripes must end exactly where the tail starts
        ShardPlan.from_widths(4 * 192 + 100, 4, 0, (128, 128), rep=100)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shard_candidates_for_the_measured_trial(world):
    p = 25_610_152
    m = StripeModel.assumed(100, world)
    c = shard_candidates(p, world, m)
    assert c[0] == plan_shards(p, world, m)  # the model's choice first
    assert any(rep == 0 for _, rep in c)  # the plan without replicated work is always tried
    assert len(set((tuple(w), r) for w, r in c)) == len(c)  # distinct
    for w, rep in c:
        plan = ShardPlan.from_widths(p, world, 0, w, rep=rep)
        assert plan.full_cols >= p
    assert shard_candidates(p, 1, m) == [plan_shards(p, 1, m)]
    # the serial plan (one stripe, no tail: no overlap to lose to contention) is always tried,
    # and so is the plan of the model with the measured contention terms
    lc = -(-p // world)
    assert ((-(-lc // ALIGN) * ALIGN,), 0) in [(tuple(w), r) for w, r in c]
    from flearn_amd.dist import CONTENTION_PRIOR
    cp = plan_shards(p, world, m.with_contention(*CONTENTION_PRIOR))
    assert (tuple(cp[0]), cp[1]) in [(tuple(w), r) for w, r in c]


def test_makespan_contention_terms():
    """c_r / c_g: reduces that run beside a gather (every stripe after the first, and the tail)
    and gathers that run beside a reduce (all but a last gather with nothing after it) stream
    slower; zero contention is the old model exactly."""
    base = StripeModel(a_r=0.0, b_r=1.0, a_g=0.0, b_g=0.25)
    assert base.with_contention(0.0, 0.0).makespan((192, 64)) == base.makespan((192, 64))
    m = base.with_contention(0.5, 1.0)
    # reduce 0: 192; reduce 1 (beside gather 0): 64*1.5 = 96 -> 288
    # gather 0 (beside reduce 1): 48*2 = 96, 192..288; gather 1 (nothing after it): 16, 288..304
    assert m.makespan((192, 64)) == (304.0, 288.0, 16.0)
    # a replicated tail runs beside the last gather: both carry the terms
    t, red, exp = m.makespan((64,), rep=64)
    assert red == 64 + 64 * 1.5 and t == max(64 + 16 * 2.0, red)
    # one stripe, no tail: nothing overlaps
    assert m.makespan((256,)) == base.makespan((256,))
    # contention never makes a plan faster, and a fitted model carries it
    for w in ((64,), (128, 64), (64, 64, 64)):
        assert m.makespan(w)[0] >= base.makespan(w)[0]
    f = StripeModel.fit(8000, 1000, 10 + 8000 * 2, 10 + 1000 * 2, 30 + 8000 * 5, 30 + 1000 * 5, c_r=0.1, c_g=-1)
    assert (f.c_r, f.c_g) == (0.1, 0.0)
