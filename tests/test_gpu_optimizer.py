"""Fused population optimizer kernel vs the PyTorch fp32 reference (engine/optim.py)."""
import pytest
import torch

from distributedtf_amd.engine import optim as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("opt", list(O.OPT_CODES))
@pytest.mark.parametrize("reg", [None, "l1_regularizer", "l2_regularizer", "l1_l2_regularizer"])
def test_fused_optimizer_matches_reference(opt, reg):
    from distributedtf_amd import ops
    torch.manual_seed(0)
    G, P, n_reg = 3, 1000, 700
    Pp = 1024
    S = 3 * Pp + 64
    dev = "cuda"
    state = torch.randn(G, S, device=dev)
    s1i, s2i = O.slot_init_values(opt)
    state[:, Pp:2 * Pp] = state[:, Pp:2 * Pp].abs() + s1i + 0.05  # keep second-moment slots positive
    state[:, 2 * Pp:3 * Pp] = state[:, 2 * Pp:3 * Pp].abs() * 0.1 + s2i
    grads = torch.randn(G, Pp, device=dev)
    hp = {"opt_case": {"optimizer": opt, "lr": 0.01, "momentum": 0.7, "grad_decay": 0.8},
          "weight_decay": 1e-3, "regularizer": reg}
    hyper = torch.tensor([O.hyper_row(hp, 0.01 * (g + 1), 3 + g, active=(g != 1)) for g in range(G)],
                         device=dev, dtype=torch.float32)
    ref = state.clone()
    O.apply_reference(ref[:, :P], grads[:, :P], ref[:, Pp:Pp + P], ref[:, 2 * Pp:2 * Pp + P], hyper, n_reg)
    shadow = torch.zeros(G, Pp, dtype=torch.bfloat16, device=dev)
    g2 = grads.clone()
    ops.fused_optimizer(state, g2, hyper, Pp, P, n_reg, shadow=shadow, zero_grads=True)
    torch.cuda.synchronize()
    for g in range(G):
        for a, b in [(0, P), (Pp, Pp + P), (2 * Pp, 2 * Pp + P)]:
            torch.testing.assert_close(state[g, a:b], ref[g, a:b], rtol=2e-5, atol=2e-6)
    act = [0, 2]
    torch.testing.assert_close(shadow[act, :P].float(), state[act, :P].bfloat16().float())
    assert float(g2[act, :P].abs().sum()) == 0.0
    assert torch.equal(g2[1], grads[1])  # inactive member untouched
