"""The round schedule of k_tree's chain splitting (csrc/tree.hip, DESIGN.md §7
"Exact endgames"), restated as a small model: per game, virtual threads are
visited cyclically from the round's resume thread; a visit backs up the
thread's waiting batch and selects, re-selecting at once while batches come
back all terminal (search_thread.cpp:102-127); after `budget` re-selections
in a round a chain may stop (at most `cuts` times per search) and the next
round resumes it. The model checks, over random terminal patterns, that the
split schedule performs exactly the unsplit schedule's operations in the same
order and completes within steps + cuts selecting rounds (the extra rounds the
host runs). The GPU test test_chain_split_keeps_every_game_identical checks
the kernel itself against the unsplit callback path.

The adaptive extra-round count (capi.hip pick_extra_rounds) reads back the
cuts each game used, or cuts + 1 when a chain went past the budget with no
cut left (k_tree `over`); the model checks that this report is exactly the
cuts an unlimited search uses whenever it is <= the limit."""

import random


def run_schedule(T, steps, budget, cuts_max, terminal, report=None):
    """Operations ('S'elect / 'B'ackup, thread, batch) of one search; budget 0
    = the unsplit schedule (steps + 1 rounds). report: a list that receives
    the cuts the search reports (k_tree's cuts_out)."""
    X = cuts_max if budget > 0 else 0
    S = steps + X
    sel = [0] * T
    pend = [False] * T
    rp = cuts = 0
    over = False
    ops = []
    for s in range(S + 1):
        do_select, do_backup = s < S, s > 0
        if s == 0:  # a search's first round starts every thread fresh
            sel, pend, rp, cuts = [0] * T, [False] * T, 0, 0
        chain, cut_at = 0, -1
        for k in range(T):
            if cut_at >= 0:
                break
            t = (rp + k) % T
            if do_backup and pend[t]:
                ops.append(("B", t, sel[t]))
                pend[t] = False
            again = False
            while do_select and not pend[t] and sel[t] < steps:
                if again and budget > 0 and chain >= budget:
                    if cuts < cuts_max:
                        cut_at, cuts = t, cuts + 1
                        break
                    over = True  # no cut left: the chain runs on
                sel[t] += 1
                ops.append(("S", t, sel[t]))
                if terminal(t, sel[t]):
                    ops.append(("B", t, sel[t]))
                    again, chain = True, chain + 1
                else:
                    pend[t] = True
        if budget > 0 and cut_at >= 0:
            rp = cut_at
    if report is not None:
        report.append(cuts_max + 1 if over else cuts)
    return ops, sel, pend


def test_chain_split_schedule_keeps_order_and_completes():
    rng = random.Random(1)
    for _ in range(3000):
        T = rng.choice([1, 2, 3, 4])
        steps = rng.randint(1, 12)
        p = rng.random()
        tab = {(t, k): rng.random() < p for t in range(T) for k in range(1, steps + 1)}
        term = lambda t, k: tab[(t, k)]  # noqa: E731
        ref, _, _ = run_schedule(T, steps, 0, 0, term)
        budget, cuts = rng.randint(1, 8), rng.randint(1, 5)
        ops, sel, pend = run_schedule(T, steps, budget, cuts, term)
        assert ops == ref, (T, steps, budget, cuts)
        assert sel == [steps] * T and not any(pend)


def test_chain_split_needs_the_first_round_reset():
    """A split in a search's first round leaves later threads unvisited: their
    state must still start fresh (the kernel resets every thread at round 0)."""
    term = lambda t, k: True  # noqa: E731  (a terminal root: every batch is terminal)
    ops, sel, pend = run_schedule(2, 10, 1, 3, term)
    assert sel == [10, 10] and ops == run_schedule(2, 10, 0, 0, term)[0]


def test_cut_report_is_the_unlimited_demand():
    """X = cuts_max extra rounds, X from 0 (the adaptive count outside the
    endgame: budget kept, no cut allowed) up: the order of operations never
    changes, and the report is the cuts an unlimited search uses when that is
    <= X, X + 1 otherwise."""
    rng = random.Random(2)
    for _ in range(3000):
        T = rng.choice([1, 2, 3, 4])
        steps = rng.randint(1, 16)
        p = rng.random()
        tab = {(t, k): rng.random() < p for t in range(T) for k in range(1, steps + 1)}
        term = lambda t, k: tab[(t, k)]  # noqa: E731
        budget = rng.randint(1, 6)
        ref, _, _ = run_schedule(T, steps, 0, 0, term)
        need = []
        run_schedule(T, steps, budget, 64, term, need)
        X = rng.randint(0, 6)
        got = []
        ops, sel, pend = run_schedule(T, steps, budget, X, term, got)
        assert ops == ref and sel == [steps] * T and not any(pend)
        assert got[0] == (need[0] if need[0] <= X else X + 1), (T, steps, budget, X, need, got)
