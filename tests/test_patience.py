"""ccmi.train.run_phase's patience mechanism (per frame of a batch) against a restatement of
the reference's single-frame loop, enc/training/train.py:222-240 (patience check at the
start of an iteration: reload the best model and optimizer state in cosine-scheduled
phases, stop otherwise), :269-310 (validation every freq_valid iterations, record gate),
:372-373 (the best model is loaded at the end).

The batch runs on a CPU stand-in for ccmi.train.Overfitter whose "model" is one counter per
frame (params[:, 0], advanced by every update) and whose validation loss is a scripted
function of that counter, so reloads, early stops, batch shrinking and the final best state
are all observable.  No GPU needed.
"""
import math

import pytest
import torch

from ccmi import train as T


class FakeOverfitter:
    def __init__(self, tables):
        self.tables = tables                       # frame -> list of losses indexed by counter
        B = len(tables)
        self.B = B
        self.arch = T.Arch(8, 8, n_grids=2)
        self.frame = torch.arange(B, dtype=torch.float32)  # which table each row uses
        self.latents = torch.zeros(B, 4)
        self.params = torch.zeros(B, 3)
        self.params[:, 1] = self.frame
        self.targets = torch.zeros(B, 2)
        self.targets[:, 0] = self.frame
        self.m = torch.zeros(B, 7)
        self.v = torch.zeros(B, 7)
        self.steps = torch.zeros(B, dtype=torch.int32)
        self.steps_uniform = True
        self.n_steps = 0

    def reset_optimizer(self):
        self.m.zero_()
        self.v.zero_()
        self.steps.zero_()
        self.steps_uniform = True

    def validate(self, lmbda):
        out = torch.zeros(self.B, 4)
        for r in range(self.B):
            f = int(self.params[r, 1])
            c = int(self.params[r, 0])
            loss = self.tables[f][min(c, len(self.tables[f]) - 1)]
            out[r] = torch.tensor([loss, loss, 1.0, 0.0])  # rate constant: the gate reduces to loss < best
        return out

    def step(self, *a, update=True, **k):
        self.n_steps += 1
        self.params[:, 0] += 1
        self.m += 1
        self.steps += 1
        return torch.zeros(self.B, 4)

    def keep(self, idx):
        for n in ("latents", "params", "targets", "m", "v", "steps"):
            setattr(self, n, getattr(self, n)[idx].contiguous())
        self.B = int(idx.numel())

    def reset_batch(self, latents, params, targets):
        self.latents, self.params, self.targets = latents.clone(), params.clone(), targets.clone()
        self.B = latents.shape[0]
        self.m = torch.zeros(self.B, 7)
        self.v = torch.zeros(self.B, 7)
        self.steps = torch.zeros(self.B, dtype=torch.int32)


def reference_loop(table, n, freq, patience, cosine):
    """train.py:222-373 for one frame: (iterations run, final counter, reloads)."""
    c = 0
    best_loss, best_c, rec = table[0], 0, 0
    its = reloads = 0
    for cnt in range(n):
        if cnt - rec > patience:
            if cosine:
                c, rec = best_c, cnt
                reloads += 1
            else:
                break
        c += 1
        its += 1
        if (cnt + 1) % freq == 0 or cnt + 1 == n:
            loss = table[min(c, len(table) - 1)]
            # record gate train.py:280-289 with a constant rate (delta_bpp = 0 < 0.001)
            if loss < best_loss:
                best_loss, best_c, rec = loss, c, cnt
    return its, best_c, reloads


def _tables(B, L, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for b in range(B):
        # a noisy decreasing curve that plateaus at a frame-specific point
        stop = int(torch.randint(5, L, (1,), generator=g))
        base = [10.0 - 0.1 * min(i, stop) for i in range(L + 1)]
        out.append([v + 0.05 * float(torch.rand(1, generator=g)) for v in base])
    return out


@pytest.mark.parametrize("cosine", [False, True])
@pytest.mark.parametrize("freq,patience", [(1, 5), (10, 50), (3, 7)])
def test_patience_matches_reference_loop(cosine, freq, patience):
    n = 120
    tables = _tables(6, 4 * n, seed=freq * 100 + patience + int(cosine))
    of = FakeOverfitter(tables)
    ph = T.Phase(lr=1e-2, max_itr=n, freq_valid=freq, patience=patience, schedule_lr=cosine)
    best = T.run_phase(of, ph, 1e-3)
    assert of.B == len(tables)
    for b, tb in enumerate(tables):
        its, best_c, _ = reference_loop(tb, n, freq, patience, cosine)
        r = int((of.targets[:, 0] == b).nonzero()[0, 0])
        assert r == b, "batch order restored"
        assert of.phase_iterations[b] == its, (b, of.phase_iterations[b], its)
        assert int(of.params[r, 0]) == best_c, (b, int(of.params[r, 0]), best_c)
        assert math.isclose(float(best[b, 0]), tb[min(best_c, len(tb) - 1)], rel_tol=1e-6)


def test_early_stop_shrinks_batch():
    """Frames that stop leave the batch (the others step alone) and come back at the end."""
    n, freq, patience = 60, 1, 3
    flat = [5.0] * (n + 2)                       # never improves: stops after patience + 1 iterations
    improving = [5.0 - 0.01 * i for i in range(n + 2)]
    of = FakeOverfitter([flat, improving, flat])
    ph = T.Phase(max_itr=n, freq_valid=freq, patience=patience, schedule_lr=False)
    T.run_phase(of, ph, 1e-3)
    assert of.phase_iterations == [patience + 1, n, patience + 1]
    assert of.n_steps == n                       # the improving frame kept stepping alone
    assert of.B == 3 and [int(v) for v in of.targets[:, 0]] == [0, 1, 2]
    assert [int(v) for v in of.params[:, 0]] == [0, n, 0]


def test_cosine_reload_restores_optimizer_state():
    n, freq, patience = 40, 1, 4
    # improves for 3 iterations, then worse: reloads the state of counter 3 every patience + 1
    tb = [5.0, 4.9, 4.8, 4.7] + [6.0] * (n + 2)
    of = FakeOverfitter([tb])
    ph = T.Phase(max_itr=n, freq_valid=freq, patience=patience, schedule_lr=True)
    T.run_phase(of, ph, 1e-3)
    its, best_c, reloads = reference_loop(tb, n, freq, patience, True)
    assert reloads > 0 and of.phase_iterations == [its] and int(of.params[0, 0]) == best_c == 3
    assert not of.steps_uniform                  # the reload gave the frame its own Adam step
