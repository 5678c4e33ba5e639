"""Model families on CPU (torch backend): ResNet v1/v2 building/bottleneck, MNIST CNN,
LR schedule, optimizer semantics, checkpoint round trip, CSV schemas, population engine."""
import csv
import math
import os

import pytest
import torch
import torch.nn.functional as F

from distributedtf_amd.engine import optim as O
from distributedtf_amd.engine import schedule
from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.mnist import MnistArch
from distributedtf_amd.models.resnet import (ResNetArch, build_program, cifar_config, forward_reference,
                                             imagenet_config, init_kernel, init_params, regularization_loss)


def test_resnet_param_counts_match_survey():
    # ResNet-56 852 k conv+dense params (plus BN), ResNet-110 1.72 M
    a56 = ResNetArch(cifar_config(56))
    assert abs(a56.n_params - 852_000) / 852_000 < 0.01
    assert abs(ResNetArch(cifar_config(110)).n_params - 1_720_000) / 1.72e6 < 0.01
    assert abs(ResNetArch(imagenet_config(50)).n_params - 25.5e6) / 25.5e6 < 0.01
    assert abs(a56.flops_per_image() - 0.252e9) / 0.252e9 < 0.01


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("size", [8, 14])
def test_resnet_forward_backward_cpu(version, size):
    arch = ResNetArch(cifar_config(size, version))
    p, r = arch.init_params("he_init", 0)
    p.requires_grad_(True)
    x = torch.randn(4, 32, 32, 3)
    y = torch.randint(0, 10, (4,))
    logits = arch.forward(p, r, x, training=True)
    assert logits.shape == (4, 10)
    loss = F.cross_entropy(logits, y)
    loss.backward()
    assert torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0
    # running statistics moved away from (0, 1)
    assert r.abs().sum() > 0


def test_bottleneck_imagenet_small_forward():
    cfg = imagenet_config(50, 2, num_classes=11, image_size=64)
    arch = ResNetArch(cfg)
    p, r = arch.init_params(None, 1)
    out = arch.forward(p, r, torch.randn(2, 64, 64, 3), training=True)
    assert out.shape == (2, 11)


def test_resnet_v2_block_matches_torch_modules():
    """v2 building block (BN->ReLU->conv, projection on the pre-activation) vs nn modules."""
    cfg = cifar_config(8, 2)
    prog = build_program(cfg)
    p, r = init_params(prog, "glorot_normal", 3)
    x = torch.randn(2, 32, 32, 3)
    out = forward_reference(prog, p, r.clone(), x, training=True)
    # independent re-implementation with torch.nn layers
    def conv(i):
        c = prog.convs[i]
        m = torch.nn.Conv2d(c.cin, c.cout, c.k, c.stride, (c.k - 1) // 2, bias=False)
        m.weight.data = p[c.off:c.off + c.numel].view(c.cout, c.k, c.k, c.cin).permute(0, 3, 1, 2).clone()
        return m

    def bn(i):
        b = prog.bns[i]
        m = torch.nn.BatchNorm2d(b.c, eps=1e-5, momentum=0.003)
        m.weight.data = p[b.gamma_off:b.gamma_off + b.c].clone()
        m.bias.data = p[b.beta_off:b.beta_off + b.c].clone()
        return m.train()
    h = conv(prog.stem)(x.permute(0, 3, 1, 2))
    for blk in prog.blocks:
        pre = F.relu(bn(blk.bns[0])(h))
        sc = conv(blk.proj)(pre) if blk.proj is not None else h
        t = conv(blk.convs[0])(pre)
        t = conv(blk.convs[1])(F.relu(bn(blk.bns[1])(t)))
        h = t + sc
    h = F.relu(bn(prog.final_bn)(h)).mean(dim=(2, 3))
    w = p[prog.dense_w_off:prog.dense_w_off + 640].view(10, 64)
    ref = h @ w.t() + p[prog.dense_b_off:prog.dense_b_off + 10]
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("init", ["glorot_normal", "he_init", "orthogonal", None])
def test_initializers(init):
    g = torch.Generator().manual_seed(0)
    w = init_kernel((64, 3, 3, 16), init, g)
    fan_in = 144
    if init == "he_init":
        assert abs(w.std().item() - math.sqrt(2.0 / fan_in)) < 0.02
    if init == "orthogonal":
        m = w.reshape(64, -1)
        torch.testing.assert_close(m @ m.t(), torch.eye(64), atol=1e-4, rtol=1e-4)
    assert w.abs().max() < 1.0


def test_regularization_loss():
    p = torch.tensor([1.0, -2.0, 3.0])
    assert regularization_loss(2, p, "l2_regularizer", 0.1).item() == pytest.approx(0.1 * 0.5 * 5)
    assert regularization_loss(2, p, "l1_regularizer", 0.1).item() == pytest.approx(0.3)
    assert regularization_loss(2, p, "None", 0.1).item() == 0.0


def test_cifar_lr_schedule():
    hp = {"opt_case": {"lr": 0.1}, "batch_size": 128, "decay_steps": 0, "decay_rate": 0.1}
    assert schedule.cifar_lr(hp, 0) == pytest.approx(0.1)
    assert schedule.cifar_lr(hp, 10 ** 6) == pytest.approx(0.1)
    hp.update(decay_steps=20, decay_rate=0.5, batch_size=256)
    b, v = schedule.cifar_boundaries(hp)
    # ceil(100/20)-1 = 4 boundaries at 50,100,150,200 epochs of 50000/256 steps
    assert len(b) == 4 and b[0] == int(50000 / 256 * 50)
    assert v[0] == pytest.approx(0.2) and v[1] == pytest.approx(0.1) and v[4] == pytest.approx(0.2 * 0.5 ** 4)
    assert schedule.cifar_lr(hp, b[0]) == pytest.approx(v[0])
    assert schedule.cifar_lr(hp, b[0] + 1) == pytest.approx(v[1])
    hp["decay_steps"] = 100
    assert schedule.cifar_boundaries(hp)[1] == [0.2, 0.2]


@pytest.mark.parametrize("opt", list(O.OPT_CODES))
def test_optimizer_reference_semantics(opt):
    """One step of each TF1 optimizer rule against a hand-written scalar version."""
    w0, g0 = 0.5, 0.2
    lr, mu, dec = 0.1, 0.9, 0.9
    s1, s2 = O.slot_init_values(opt)
    params = torch.tensor([[w0]])
    a = torch.tensor([[s1]])
    b = torch.tensor([[s2]])
    hp = {"opt_case": {"optimizer": opt, "lr": lr, "momentum": mu, "grad_decay": dec}}
    hyper = torch.tensor([O.hyper_row(hp, lr, 1)])
    O.apply_reference(params, torch.tensor([[g0]]), a, b, hyper, 0)
    if opt == "gd":
        exp = w0 - lr * g0
    elif opt == "Momentum":
        exp = w0 - lr * g0
    elif opt == "Adam":
        m, v = 0.1 * g0, 0.001 * g0 * g0
        exp = w0 - lr * math.sqrt(1 - 0.999) / (1 - 0.9) * m / (math.sqrt(v) + 1e-8)
    elif opt == "Adagrad":
        exp = w0 - lr * g0 / math.sqrt(0.1 + g0 * g0)
    elif opt == "Adadelta":
        acc = 0.05 * g0 * g0
        upd = math.sqrt(1e-8) / math.sqrt(acc + 1e-8) * g0
        exp = w0 - lr * upd
    else:
        ms = dec * 1.0 + (1 - dec) * g0 * g0
        exp = w0 - lr * g0 / math.sqrt(ms + 1e-10)
    assert params.item() == pytest.approx(exp, rel=1e-5)


def test_population_engine_state_rows_and_import():
    arch = ResNetArch(cifar_config(8))
    eng = PopulationEngine(arch, 3, "cpu")
    hp = {"opt_case": {"optimizer": "Momentum", "lr": 0.1, "momentum": 0.9}, "initializer": "he_init",
          "batch_size": 4, "regularizer": "l2_regularizer", "weight_decay": 1e-4}
    s0 = eng.add_member(None, hp, 1)
    s1 = eng.add_member(None, hp, 2)
    assert not torch.equal(eng.params[s0], eng.params[s1])
    x = torch.randn(4, 32, 32, 3)
    y = torch.randint(0, 10, (4,))
    losses = eng.train_step([s0, s1], [(x, y), (x, y)], [hp, hp], [0.1, 0.1])
    assert losses.shape == (2,) and torch.isfinite(losses).all()
    assert eng.host_step[s0] == 1 and eng.step_col()[s0].item() == 1.0
    # exploit copy = one row copy; step counter travels with the state
    eng.state[s1].copy_(eng.state[s0])
    eng.on_state_imported(s1, eng.host_step[s0])
    assert eng.host_step[s1] == 1 and torch.equal(eng.params[s1], eng.params[s0])
    assert eng.slot1[s0].abs().sum() > 0  # momentum slot populated


def test_mnist_arch_forward():
    a = MnistArch()
    p, r = a.init_params("glorot_normal", 0)
    out = a.forward(p, r, torch.rand(3, 28, 28, 1) * 255, training=True)
    assert out.shape == (3, 10) and a.n_params == 3_274_634


def test_cifar_model_csv_and_checkpoint(tmp_cwd):
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    hp = {"opt_case": {"optimizer": "RMSProp", "lr": 1e-4, "momentum": 0.5, "grad_decay": 0.9},
          "decay_steps": 20, "decay_rate": 0.5, "weight_decay": 1e-4, "regularizer": "l1_regularizer",
          "initializer": "he_init", "batch_size": 4}
    m = Cifar10Model(5, hp, "savedata/model_", seed=1, resnet_size=8, device="cpu", max_train_steps=2,
                     use_synthetic_data=True)
    m.train(1, 1)
    rows = list(csv.reader(open("savedata/model_5/learning_curve.csv")))
    assert rows[0][:11] == ["epochs", "eval_accuracy", "optimizer", "learning_rate", "decay_rate", "decay_steps",
                            "initializer", "regularizer", "weight_decay", "batch_size", "model_id"]
    assert rows[0][11:13] == ["momentum", "grad_decay"]
    assert rows[1][2] == "RMSProp" and float(rows[1][3]) == 1e-4
    from distributedtf_amd.models.model_base import flush_checkpoints
    flush_checkpoints()  # checkpoints are written by a background thread
    assert os.path.isfile("savedata/model_5/model.ckpt") and os.path.isfile("savedata/model_5/checkpoint")
    before = m.export_state().clone()
    m.train(1, 2)
    assert not torch.equal(before, m.export_state())
    m.import_state(before)  # round trip through a checkpoint file
    m.save_checkpoint()
    m.import_state(torch.zeros_like(before))
    assert m.load_checkpoint() and torch.equal(m.export_state(), before)
    assert m.global_step == 2 and m.epoches_trained == 2


def test_mnist_model_csv(tmp_cwd):
    from distributedtf_amd.models.mnist_model import MNISTModel
    hp = {"opt_case": {"optimizer": "Adam", "lr": 1e-3}, "batch_size": 8, "initializer": "he_init"}
    m = MNISTModel(0, hp, "savedata/model_", seed=0, device="cpu", debug_steps=2)
    m.train(3, 3)
    assert m.epoches_trained == 1  # reference adds one per call
    rows = list(csv.reader(open("savedata/model_0/learning_curve.csv")))
    assert rows[0] == ["global_step", "eval_accuracy", "optimizer", "lr"]
