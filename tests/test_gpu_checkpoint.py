"""Checkpoint / resume: an interrupted run resumed from an SMT checkpoint is
bit-identical to the uninterrupted run (all kernels on the path are deterministic)."""
import pytest
import torch
from torch import nn

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import checkpoint
from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize, linear_lr_lambda
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
SEL_MLP = {("up_proj", 0): [(2, 0), (0, 0)], ("down_proj", 1): [(1, 2)]}
SEL_ATT = {("v_proj", 0): [(0, 1)]}


class Block(nn.Module):
    def __init__(self, i):
        super().__init__()
        self.self_attn = nn.Module()
        self.self_attn.v_proj = nn.Linear(512, 256, bias=False)
        self.mlp = nn.Module()
        self.mlp.up_proj = nn.Linear(256, 768, bias=False)
        self.mlp.down_proj = nn.Linear(768, 512, bias=False)

    def forward(self, x):
        return self.mlp.down_proj(torch.relu(self.mlp.up_proj(self.self_attn.v_proj(x))))


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.model = nn.Module()
        self.model.layers = nn.ModuleList([Block(0), Block(1)])

    def forward(self, x):
        for b in self.model.layers:
            x = b(x)
        return x


def _base():
    torch.manual_seed(0)
    net = Net().to(torch.bfloat16)
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(4.0)
    return net.to(DEV)


def _engine(net):
    smt.freeze_unselected_matrix_layer(net, SEL_MLP, SEL_ATT)
    smt.convert_linear_layer_to_matrix_sparsity(net, SEL_MLP, SEL_ATT)
    groups = smt.get_optimizer_sparse_grouped_parameters(net, 0.01, 2e-3)
    opt = SMTFusedAdam(groups, lr=2e-3, betas=(0.9, 0.95))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, linear_lr_lambda(1, 10))
    eng, _, _, _ = initialize(model=net, optimizer=opt, config={"gradient_clipping": 1.0}, lr_scheduler=sched)
    return eng


def _step(eng, i):
    x = torch.randn(2, 32, 512, generator=torch.Generator().manual_seed(100 + i)).bfloat16().to(DEV)
    loss = (eng(x).float() ** 2).mean()
    eng.backward(loss)
    eng.step()
    return loss.item()


def test_resume_is_bit_identical(tmp_path):
    base_sd = {k: v.clone() for k, v in _base().state_dict().items()}
    a = _engine(_base())
    for i in range(4):
        _step(a, i)
    b = _engine(_base())
    for i in range(2):
        _step(b, i)
    b.save_checkpoint(str(tmp_path), tag="step2", client_state={"epoch": 0})
    del b
    net = _base()
    net.load_state_dict(base_sd)
    checkpoint.restore_model(net, str(tmp_path / "step2"))
    c = _engine_restored(net)
    assert c.load_checkpoint(str(tmp_path), tag="step2") == {"epoch": 0}
    for i in range(2, 4):
        _step(c, i)
    torch.cuda.synchronize()
    for ta, tc in zip(a.tile_groups, c.tile_groups):
        assert torch.equal(ta.master, tc.master) and torch.equal(ta.exp_avg_sq, tc.exp_avg_sq)
    for (na, pa), (nc, pc) in zip(a.module.named_parameters(), c.module.named_parameters()):
        assert na == nc and torch.equal(pa, pc), na
    assert c.global_steps == 4 and c.lr_scheduler.last_epoch == a.lr_scheduler.last_epoch


def _engine_restored(net):
    groups = smt.get_optimizer_sparse_grouped_parameters(net, 0.01, 2e-3)
    opt = SMTFusedAdam(groups, lr=2e-3, betas=(0.9, 0.95))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, linear_lr_lambda(1, 10))
    eng, _, _, _ = initialize(model=net, optimizer=opt, config={"gradient_clipping": 1.0}, lr_scheduler=sched)
    return eng


def test_selection_roundtrip_and_merged_export(tmp_path):
    eng = _engine(_base())
    _step(eng, 0)
    eng.save_checkpoint(str(tmp_path))
    sel_mlp, sel_att = checkpoint.read_selection(str(tmp_path))
    assert dict(sel_mlp) == SEL_MLP and dict(sel_att) == SEL_ATT
    path = str(tmp_path / "merged.safetensors")
    checkpoint.save_merged_model(eng.module, path)
    from safetensors.torch import load_file
    sd = load_file(path)
    assert not any(k.endswith("selected_weight") for k in sd)
    up = eng.module.model.layers[0].mlp.up_proj
    w = sd["model.layers.0.mlp.up_proj.weight"]
    assert torch.equal(ref.gather_tiles(w, up.index_list), up.selected_weight.detach().cpu())


def test_resume_after_full_ft_warmup(tmp_path):
    """the warm-up updates every weight before the selection. A checkpoint restored onto a
    fresh base model must not silently revert them: with the frozen weights saved it resumes
    bit-identically, without them the fingerprint check refuses the base model."""
    base_sd = {k: v.clone() for k, v in _base().state_dict().items()}

    def warm(net):
        opt = SMTFusedAdam(net.parameters(), lr=1e-2, betas=(0.9, 0.95))
        eng, _, _, _ = initialize(model=net, optimizer=opt, config={"gradient_clipping": 1.0})
        _step(eng, 99)                                  # one full fine-tuning step: every W moves
        eng.release()
        return net
    a = _engine(warm(_base()))
    for i in range(4):
        _step(a, i)
    b = _engine(warm(_base()))
    for i in range(2):
        _step(b, i)
    b.save_checkpoint(str(tmp_path), tag="full")
    b.save_checkpoint(str(tmp_path), tag="lean", include_frozen=False)
    del b
    fresh = _base()
    fresh.load_state_dict(base_sd)
    with pytest.raises(ValueError, match="frozen weights differ"):
        checkpoint.restore_model(fresh, str(tmp_path / "lean"))
    net = _base()
    net.load_state_dict(base_sd)
    checkpoint.restore_model(net, str(tmp_path / "full"))
    c = _engine_restored(net)
    c.load_checkpoint(str(tmp_path), tag="full")
    for i in range(2, 4):
        _step(c, i)
    torch.cuda.synchronize()
    for ta, tc in zip(a.tile_groups, c.tile_groups):
        assert torch.equal(ta.master, tc.master) and torch.equal(ta.exp_avg_sq, tc.exp_avg_sq)
    for (na, pa), (nc, pc) in zip(a.module.named_parameters(), c.module.named_parameters()):
        assert na == nc and torch.equal(pa, pc), na


class GroupBlock(nn.Module):
    """q/k/v and gate/up read one input each: the fp8 path turns them into groups whose members'
    W are row slices of one joint buffer (fp8.Fp8Group)."""

    def __init__(self):
        super().__init__()
        self.self_attn = nn.Module()
        self.self_attn.q_proj = nn.Linear(512, 512, bias=False)
        self.self_attn.k_proj = nn.Linear(512, 256, bias=False)
        self.self_attn.v_proj = nn.Linear(512, 256, bias=False)
        self.mlp = nn.Module()
        self.mlp.gate_proj = nn.Linear(512, 768, bias=False)
        self.mlp.up_proj = nn.Linear(512, 768, bias=False)
        self.mlp.down_proj = nn.Linear(768, 512, bias=False)

    def forward(self, x):
        a = self.self_attn
        h = a.q_proj(x) + torch.cat([a.k_proj(x), a.v_proj(x)], -1)
        return self.mlp.down_proj(torch.relu(self.mlp.gate_proj(h)) * self.mlp.up_proj(h))


class GroupNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.model = nn.Module()
        self.model.layers = nn.ModuleList([GroupBlock()])

    def forward(self, x):
        return self.model.layers[0](x)


G_MLP = {("gate_proj", 0): [(1, 0)], ("down_proj", 0): [(0, 2)]}
G_ATT = {("q_proj", 0): [(0, 1)], ("v_proj", 0): [(0, 0)]}


def _gbase():
    torch.manual_seed(1)
    net = GroupNet().to(torch.bfloat16)
    with torch.no_grad():
        for p in net.parameters():
            p.mul_(4.0)
    return net.to(DEV)


def _gengine(net, convert=True):
    if convert:
        smt.freeze_unselected_matrix_layer(net, G_MLP, G_ATT)
        smt.convert_linear_layer_to_matrix_sparsity(net, G_MLP, G_ATT)
    groups = smt.get_optimizer_sparse_grouped_parameters(net, 0.01, 2e-3)
    opt = SMTFusedAdam(groups, lr=2e-3, betas=(0.9, 0.95))
    eng, _, _, _ = initialize(model=net, optimizer=opt, config={"gradient_clipping": 1.0, "fp8_linears": True})
    return eng


def test_fp8_group_resume_is_bit_identical(tmp_path):
    """The fp8 path's grouped weights (joint buffers, re-quantised after every step) survive a save /
    restore: the resumed run equals the uninterrupted one bit for bit."""
    from sparse_matrix_tuning_amd.fp8 import Fp8Group
    base_sd = {k: v.clone() for k, v in _gbase().state_dict().items()}
    a = _gengine(_gbase())
    attn = a.module.model.layers[0].self_attn
    grp = attn.q_proj.weight._smt_fp8.group
    assert isinstance(grp, Fp8Group) and grp._cat() is grp.joint      # members alias the joint buffer
    for i in range(4):
        _step(a, i)
    b = _gengine(_gbase())
    for i in range(2):
        _step(b, i)
    b.save_checkpoint(str(tmp_path), tag="s2")
    del b
    net = _gbase()
    net.load_state_dict(base_sd)
    checkpoint.restore_model(net, str(tmp_path / "s2"))
    c = _gengine(net, convert=False)
    c.load_checkpoint(str(tmp_path), tag="s2")
    for i in range(2, 4):
        _step(c, i)
    torch.cuda.synchronize()
    for ta, tc in zip(a.tile_groups, c.tile_groups):
        assert torch.equal(ta.master, tc.master) and torch.equal(ta.exp_avg_sq, tc.exp_avg_sq)
    for (na, pa), (nc, pc) in zip(a.module.named_parameters(), c.module.named_parameters()):
        assert na == nc and torch.equal(pa, pc), na


FP16_CFG = {"gradient_clipping": 1.0, "fp16": {"enabled": True, "loss_scale_window": 2, "initial_scale_power": 24}}


def _engine16(net, convert=True, cfg=FP16_CFG):
    if convert:
        smt.freeze_unselected_matrix_layer(net, SEL_MLP, SEL_ATT)
        smt.convert_linear_layer_to_matrix_sparsity(net, SEL_MLP, SEL_ATT)
    groups = smt.get_optimizer_sparse_grouped_parameters(net, 0.01, 2e-3)
    opt = SMTFusedAdam(groups, lr=2e-3, betas=(0.9, 0.95))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, linear_lr_lambda(1, 10))
    eng, _, _, _ = initialize(model=net, optimizer=opt, config=cfg, lr_scheduler=sched)
    return eng


def _step16(eng, i):
    x = torch.randn(2, 32, 512, generator=torch.Generator().manual_seed(100 + i)).half().to(DEV)
    loss = (eng(x).float() ** 2).mean()
    eng.backward(loss)
    eng.step()


def test_fp16_resume_keeps_the_loss_scale(tmp_path):
    """The reference's --dtype fp16 under the engine: an fp16 run interrupted after steps that
    overflowed and resumed from its checkpoint continues the dynamic loss scale's schedule (scale,
    tolerance, iteration, last overflow) and is bit-identical to the uninterrupted run; resuming
    it without the fp16 config is refused."""
    def base16():
        return _base().half()
    base_sd = {k: v.clone() for k, v in base16().state_dict().items()}
    a = _engine16(base16())
    for i in range(8):
        _step16(a, i)
    b = _engine16(base16())
    for i in range(4):
        _step16(b, i)
    assert b.skipped_steps >= 1                           # the first steps overflow at 2**24
    b.save_checkpoint(str(tmp_path), tag="s4")
    saved = dict(b.loss_scaler.state_dict())
    del b
    net = base16()
    net.load_state_dict(base_sd)
    checkpoint.restore_model(net, str(tmp_path / "s4"))
    c = _engine16(net, convert=False)
    c.load_checkpoint(str(tmp_path), tag="s4")
    assert c.loss_scaler.state_dict() == saved
    for i in range(4, 8):
        _step16(c, i)
    torch.cuda.synchronize()
    assert c.loss_scaler.state_dict() == a.loss_scaler.state_dict()
    assert c.skipped_steps == a.skipped_steps and c.global_steps == a.global_steps == 8
    for ta, tc in zip(a.tile_groups, c.tile_groups):
        assert ta.step == tc.step
        assert torch.equal(ta.master, tc.master) and torch.equal(ta.exp_avg_sq, tc.exp_avg_sq)
    for (na, pa), (nc, pc) in zip(a.module.named_parameters(), c.module.named_parameters()):
        assert na == nc and pa.dtype == torch.float16 and torch.equal(pa, pc), na
    net = base16()
    net.load_state_dict(base_sd)
    checkpoint.restore_model(net, str(tmp_path / "s4"))
    d = _engine16(net, convert=False, cfg={"gradient_clipping": 1.0})
    with pytest.raises(ValueError, match="loss scale"):
        d.load_checkpoint(str(tmp_path), tag="s4")
