"""TF tensor-bundle writer (utils/tf_bundle.py) and member export in the reference's checkpoint format
(SURVEY.md §2.7 / §5.4): byte-identical re-serialisation of every TF-written fixture shipped with the
reference, and ResNet / MNIST members exported under the reference's TF variable names and layouts."""
import glob
import os

import numpy as np
import pytest
import torch

from distributedtf_amd.utils import tf_bundle as tb

REF = "/root/reference/resnet/official/utils/testing/reference_data"
FIXTURES = sorted(glob.glob(os.path.join(REF, "**", "model.ckpt.index"), recursive=True))


def test_crc32c_vectors():
    assert tb.crc32c(b"123456789") == 0xE3069283
    assert tb._crc32c_py(b"123456789") == 0xE3069283
    data = bytes(range(256)) * 33
    assert tb.crc32c(data) == tb._crc32c_py(data)


@pytest.mark.skipif(not FIXTURES, reason="reference fixtures not mounted")
@pytest.mark.parametrize("index", FIXTURES, ids=lambda p: os.path.basename(os.path.dirname(p)))
def test_writer_reproduces_tf_saver_bytes(index, tmp_path):
    prefix = index[:-len(".index")]
    tensors = tb.load_bundle(prefix)
    out = str(tmp_path / "model.ckpt")
    tb.write_bundle(out, tensors)
    assert open(out + ".index", "rb").read() == open(index, "rb").read()
    data = glob.glob(prefix + ".data-*")[0]
    assert open(out + ".data-00000-of-00001", "rb").read() == open(data, "rb").read()


def _hp(opt):
    return {"opt_case": {"optimizer": opt, "lr": 1e-3, "momentum": 0.9, "grad_decay": 0.9}, "decay_steps": 0,
            "decay_rate": 1.0, "weight_decay": 0.0, "regularizer": "None", "initializer": "he_init", "batch_size": 4}


@pytest.mark.parametrize("opt,slots", [("Momentum", ["Momentum"]), ("Adam", ["Adam", "Adam_1"]),
                                       ("RMSProp", ["RMSProp", "RMSProp_1"]), ("gd", [])])
def test_resnet_member_export(tmp_cwd, opt, slots):
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    m = Cifar10Model(3, _hp(opt), "savedata/model_", seed=1, resnet_size=8, device="cpu", max_train_steps=2,
                     use_synthetic_data=True)
    m.train(1, 1)
    prefix = m.export_tf_checkpoint()
    assert prefix.endswith("model_3/model.ckpt-2")
    t = tb.load_bundle(prefix)
    prog = m.arch.prog
    assert int(t["global_step"]) == 2 and t["global_step"].dtype == np.int64
    # kernels: HWIO, named in creation order
    c = prog.convs[1]
    k = t["resnet_model/conv2d_1/kernel"]
    assert k.shape == (c.k, c.k, c.cin, c.cout)
    w = m.engine.params[m.slot, c.off:c.off + c.numel].view(c.cout, c.k, c.k, c.cin).permute(1, 2, 3, 0)
    np.testing.assert_array_equal(k, w.numpy())
    assert t["resnet_model/dense/kernel"].shape == (64, 10)
    nb = len(prog.bns)
    assert "resnet_model/batch_normalization_%d/moving_variance" % (nb - 1) in t
    for s in slots:
        assert "resnet_model/conv2d/kernel/" + s in t
    if opt == "Adam":
        assert t["beta1_power"] == pytest.approx(0.9 ** 2)
    assert 'model_checkpoint_path: "model.ckpt-2"' in open("savedata/model_3/checkpoint").read()


def test_mnist_member_export_names(tmp_cwd):
    from distributedtf_amd.models.mnist_model import MNISTModel
    m = MNISTModel(0, _hp("Momentum"), "savedata/model_", seed=1, device="cpu", max_train_steps=1,
                   use_synthetic_data=True, eval_every_round=False)
    t = m.tf_variables()
    assert t["conv2d/kernel"].shape == (5, 5, 1, 32) and t["conv2d_1/kernel"].shape == (5, 5, 32, 64)
    assert t["dense/kernel"].shape == (3136, 1024) and t["dense_1/kernel"].shape == (1024, 10)
    assert "dense_1/bias/Momentum" in t


@pytest.mark.parametrize("opt", ["Momentum", "Adam"])
def test_tf_checkpoint_round_trip_into_member(tmp_cwd, opt):
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    a = Cifar10Model(0, _hp(opt), "savedata/model_", seed=1, resnet_size=8, device="cpu", max_train_steps=3,
                     use_synthetic_data=True)
    a.train(1, 1)
    prefix = a.export_tf_checkpoint()
    b = Cifar10Model(1, _hp(opt), "savedata/model_", seed=2, resnet_size=8, device="cpu", use_synthetic_data=True)
    assert not torch.equal(a.export_state(), b.export_state())
    n = b.import_tf_checkpoint(prefix)
    assert n > 0 and b.global_step == 3
    torch.testing.assert_close(b.export_state(), a.export_state(), rtol=0, atol=0)


def test_exploit_destination_gets_winner_tf_bundle(tmp_cwd):
    """with --tf_checkpoint an exploit destination's directory must hold the WINNER's TF checkpoint
    (the reference copies the files: pbt_cluster.py:145-147) -- the bundle is re-exported from the imported state,
    the loser's stale bundle is removed, and the ``checkpoint`` state file names the new bundle."""
    import glob as _glob
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    from distributedtf_amd.models.engine_model import EngineModel
    from distributedtf_amd.parallel.comm import SingleComm
    from distributedtf_amd.pbt.cluster import SPMDPopulation
    EngineModel.reset_engines()
    hps = [dict(_hp("Momentum"), batch_size=4 + i) for i in range(4)]
    pop = SPMDPopulation(4, SingleComm(), Cifar10Model, epochs_per_round=1, seed=3, verbose=False, hparams=hps,
                         model_kwargs=dict(resnet_size=8, device="cpu", backend="torch", use_synthetic_data=True,
                                           max_train_steps=2 + 0, tf_checkpoint=True))
    pop.train(1)
    (p,) = pop.last_plan
    members = pop.worker.members_by_id()
    dst = members[p.dst_id]
    bundles = _glob.glob(os.path.join(dst.save_dir, "model.ckpt-*.index"))
    assert len(bundles) == 1, bundles
    state = open(os.path.join(dst.save_dir, "checkpoint")).read()
    step = members[p.src_id].global_step
    assert 'model_checkpoint_path: "model.ckpt-%d"' % step in state
    fresh = Cifar10Model(9, _hp("Momentum"), "savedata/model_", seed=7, resnet_size=8, device="cpu", backend="torch",
                         use_synthetic_data=True)
    fresh.import_tf_checkpoint(bundles[0][:-len(".index")])
    torch.testing.assert_close(fresh.export_state(), dst.export_state(), rtol=0, atol=0)
    torch.testing.assert_close(dst.export_state(), members[p.src_id].export_state(), rtol=0, atol=0)
