"""Solver and Architect policy/value networks (reference: heist_architect/networks.py).

Same module tree, parameter names and shapes as the reference, so state_dicts and
torch.save checkpoints interchange (networks.py:13-239).  They run on PyTorch-ROCm
(MIOpen convolutions / hipBLASLt GEMMs on MFMA).  Differences are in execution only:
  * SolverNetwork evaluates its single-step LSTM as one fused gate GEMM pair instead of
    an nn.LSTM sequence call (same weights, same math), and accepts channels-last
    [N,3,R,C] batches from the batched environment;
  * ArchitectNetwork.generate_layouts samples N layouts at once and decodes them on the
    GPU (heist_architect_decode) straight into the environment's layout arrays.
"""
from typing import Optional, Tuple

import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F


def _conv_nobias(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 convolution without its bias (MIOpen), channels-last out."""
    y = torch.ops.aten.convolution(x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1)
    return y.contiguous(memory_format=torch.channels_last)


def _conv_bwd(g: torch.Tensor, x: torch.Tensor, w: torch.Tensor, need_input: bool):
    gi, gw, _ = torch.ops.aten.convolution_backward(g, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                    [need_input, True, False])
    return gi, gw


class _BackboneF32(torch.autograd.Function):
    """SolverNetwork's conv stack (networks.py:93-100: relu(conv1) -> relu(conv2) ->
    relu(conv3) -> AdaptiveAvgPool2d(4, 4), flattened) in fp32 with the tail of every layer
    fused into one pass (csrc/heist_train.hip): the convolutions run on MIOpen WITHOUT their
    bias, then one kernel adds the bias and applies ReLU in place (conv3's also pools); the
    backward applies ReLU's mask (and, for conv3, the pool's gradient) in one pass that also
    forms the bias gradient, and calls MIOpen's data / weight gradients.  Same arithmetic as
    the unfused torch ops up to the order of the pool and bias-gradient sums.  Returns the
    pooled features [B, C * 16]."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        from . import _native as nat
        L, st = nat.lib(), nat.stream(x.device)
        n, _, R, C = x.shape
        x = x.contiguous(memory_format=torch.channels_last)
        a1 = _conv_nobias(x, w1)
        nat.check(L.heist_bias_relu_nhwc(nat.ptr_nhwc(a1), nat.ptr(b1), n * R * C, a1.shape[1], st), "heist_bias_relu_nhwc")
        a2 = _conv_nobias(a1, w2)
        nat.check(L.heist_bias_relu_nhwc(nat.ptr_nhwc(a2), nat.ptr(b2), n * R * C, a2.shape[1], st), "heist_bias_relu_nhwc")
        a3 = _conv_nobias(a2, w3)
        feat = torch.empty(n, a3.shape[1] * 16, dtype=torch.float32, device=x.device)
        nat.check(L.heist_bias_relu_pool_nhwc(nat.ptr_nhwc(a3), nat.ptr(b3), n, R, C, a3.shape[1], nat.ptr(feat), st),
                  "heist_bias_relu_pool_nhwc")
        ctx.save_for_backward(x, w1, w2, w3, a1, a2, a3)
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        from . import _native as nat
        L = nat.lib()
        x, w1, w2, w3, a1, a2, a3 = ctx.saved_tensors
        st = nat.stream(x.device)
        n, _, R, C = x.shape
        dfeat = dfeat.contiguous()
        part = torch.empty(n, 64, dtype=torch.float32, device=x.device)
        db3 = torch.empty(a3.shape[1], dtype=torch.float32, device=x.device)
        d3 = torch.empty_like(a3, memory_format=torch.channels_last)
        nat.check(L.heist_pool_relu_bwd_nhwc(nat.ptr(dfeat), nat.ptr_nhwc(a3), n, R, C, a3.shape[1], nat.ptr_nhwc(d3),
                                             nat.ptr(part), nat.ptr(db3), st), "heist_pool_relu_bwd_nhwc")
        g2, dw3 = _conv_bwd(d3, a2, w3, True)
        g2 = g2.contiguous(memory_format=torch.channels_last)
        db2 = torch.empty(a2.shape[1], dtype=torch.float32, device=x.device)
        nat.check(L.heist_relu_bwd_nhwc(nat.ptr_nhwc(g2), nat.ptr_nhwc(a2), n, R * C, a2.shape[1], nat.ptr(part), nat.ptr(db2), st),
                  "heist_relu_bwd_nhwc")
        g1, dw2 = _conv_bwd(g2, a1, w2, True)
        g1 = g1.contiguous(memory_format=torch.channels_last)
        db1 = torch.empty(a1.shape[1], dtype=torch.float32, device=x.device)
        nat.check(L.heist_relu_bwd_nhwc(nat.ptr_nhwc(g1), nat.ptr_nhwc(a1), n, R * C, a1.shape[1], nat.ptr(part), nat.ptr(db1), st),
                  "heist_relu_bwd_nhwc")
        _, dw1 = _conv_bwd(g1, x, w1, False)
        return None, dw1, db1, dw2, db2, dw3, db3


_TC_QUEUES = {}
_TC_FRAGS = {}  # (id(conv weight), mode) -> (weakref to the weight, its _version, packed fragments)


def _tc_frag(layer: int, mode: int, w: torch.Tensor, st) -> torch.Tensor:
    """The MFMA fragment pack of conv weight w (heist_train_conv_pack), re-packed only when w
    changed (its version counter: an optimizer step) -- a rollout's ticks reuse one pack."""
    from . import _native as nat
    key = (id(w), mode)
    hit = _TC_FRAGS.get(key)
    if hit is not None and hit[0]() is w and hit[1] == w._version:
        return hit[2]
    L = nat.lib()
    f = torch.empty(L.heist_train_conv_frag_floats(layer, mode), dtype=torch.float32, device=w.device)
    wc = w.detach().contiguous()
    nat.check(L.heist_train_conv_pack(layer, mode, nat._vp(wc.data_ptr()), nat._vp(f.data_ptr()), st),
              "heist_train_conv_pack")
    if len(_TC_FRAGS) > 64:  # entries of weights that died (a weakref gone dead)
        for k in [k for k, v in _TC_FRAGS.items() if v[0]() is None]:
            del _TC_FRAGS[k]
    _TC_FRAGS[key] = (weakref.ref(w), w._version, f)
    return f


def _tc_queues(dev) -> torch.Tensor:
    """8 work-queue counter pairs per device (one per launch site of _BackboneMFMA32), zero
    between launches: each kernel's last workgroup resets its pair."""
    q = _TC_QUEUES.get(dev)
    if q is None:
        q = _TC_QUEUES[dev] = torch.zeros(16, dtype=torch.int32, device=dev)
    return q


def _tc_act(n, R, C, ch, dev) -> torch.Tensor:
    """[n][R][C][ch + 4] activation buffer (the 4 pad words per position are never read)."""
    return torch.empty((n, R, C, ch + 4 if ch > 4 else 4), dtype=torch.float32, device=dev)


def _tc_mask(n, R, C, ch, dev) -> torch.Tensor:
    """[n][R][C][ch / 4] ReLU mask bits (uint8: bit r of byte k = channel 4 k + r > 0)."""
    return torch.empty((n, R, C, ch // 4), dtype=torch.uint8, device=dev)


def _wgrad_splitk(g: torch.Tensor, x: torch.Tensor, chunks: int = 16) -> torch.Tensor:
    """dW = g^T x over many rows and few outputs (the Solver's fc / LSTM / head weight
    gradients over a 16,384-row minibatch): the rows in `chunks` slices as one batched GEMM, the
    partials summed in slice order -- one GEMM of this shape fills a fraction of the chip
    (480 -> 172 us for the update's five, profiles/r06zs_dw_splitk.log); the result differs from
    the single GEMM's only by the order of the fp32 sums."""
    m = g.shape[0]
    step = m // chunks
    main = step * chunks
    gb = g[:main].reshape(chunks, step, g.shape[1])
    xb = x[:main].reshape(chunks, step, x.shape[1])
    dw = torch.bmm(gb.transpose(1, 2), xb).sum(0)
    if main < m:
        dw = dw + g[main:].t() @ x[main:]
    return dw


class _LinearSplitK(torch.autograd.Function):
    """F.linear whose weight gradient is _wgrad_splitk (input gradient and bias gradient as
    autograd forms them: g @ W, g summed over rows)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous()
        dx = g @ w if ctx.needs_input_grad[0] else None
        dw = _wgrad_splitk(g, x.contiguous()) if ctx.needs_input_grad[1] else None
        db = g.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


def _linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    """F.linear; in an fp32 training forward on a HIP device over >= 4,096 rows, with the
    split-K weight gradient (HEIST_SPLITK_WGRAD=0 turns it off)."""
    import os
    if (torch.is_grad_enabled() and w.requires_grad and x.is_cuda and x.dim() == 2 and x.shape[0] >= 4096
            and x.dtype == torch.float32 and w.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")
            and os.environ.get("HEIST_SPLITK_WGRAD", "1") != "0"):
        return _LinearSplitK.apply(x, w, b)
    return F.linear(x, w, b)


def _mlp_head(seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """Linear, ReLU, Linear (the policy / value heads) on _linear."""
    return _linear(F.relu(_linear(x, seq[0].weight, seq[0].bias)), seq[2].weight, seq[2].bias)


class _BackboneMFMA32(torch.autograd.Function):
    """SolverNetwork's conv stack (networks.py:93-100) forward and backward on the hand-written
    fp32-MFMA kernels (csrc/heist_train_conv.hip, heist_train_* in include/heist.h): conv1-3
    with bias + ReLU fused in their epilogues (which also write each ReLU mask as bits), the
    4x4 adaptive pool; backward the pool's gradient with conv3's mask, the data gradients of
    conv3 and conv2 with the masks of their inputs fused, and the weight + bias gradients of all
    three (fixed-order sums).
    Exact fp32 (MFMA f32 = an fmaf chain); differs from torch / MIOpen by summation order.
    Returns the pooled features [B, 1024]."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        from . import _native as nat
        L, st = nat.lib(), nat.stream(x.device)
        n, _, R, C = x.shape
        dev = x.device
        q = _tc_queues(dev)
        P = lambda t: nat._vp(t.data_ptr())  # noqa: E731
        frags = [_tc_frag(layer, 0, w, st) for layer, w in ((1, w1), (2, w2), (3, w3))]
        x4 = _tc_act(n, R, C, 3, dev)
        s = x.stride()
        nat.check(L.heist_train_obs_nhwc4(P(x), n, R, C, s[0], s[1], s[2], s[3], P(x4), st), "heist_train_obs_nhwc4")
        a1, a2, a3 = _tc_act(n, R, C, 32, dev), _tc_act(n, R, C, 64, dev), _tc_act(n, R, C, 64, dev)
        m1, m2, m3 = _tc_mask(n, R, C, 32, dev), _tc_mask(n, R, C, 64, dev), _tc_mask(n, R, C, 64, dev)
        for k, (layer, xi, yo, b, mo) in enumerate(((1, x4, a1, b1, m1), (2, a1, a2, b2, m2), (3, a2, a3, b3, m3))):
            nat.check(L.heist_train_conv(layer, 0, P(xi), n, R, C, P(frags[k]), P(b.detach().contiguous()), P(mo),
                                         P(yo), P(q[2 * k:]), st), "heist_train_conv")
        feat = torch.empty(n, 1024, dtype=torch.float32, device=dev)
        nat.check(L.heist_train_pool(P(a3), n, R, C, P(feat), st), "heist_train_pool")
        del a3  # only its pool and its mask bits are needed later
        ctx.save_for_backward(x4, a1, a2, m1, m2, m3, w2, w3)
        ctx.frags = frags  # the forward's packs stay alive until the kernels that read them ran
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        from . import _native as nat
        L = nat.lib()
        x4, a1, a2, m1, m2, m3, w2, w3 = ctx.saved_tensors
        n, R, C = x4.shape[0], x4.shape[1], x4.shape[2]
        dev = x4.device
        st = nat.stream(dev)
        q = _tc_queues(dev)
        P = lambda t: nat._vp(t.data_ptr())  # noqa: E731
        dfeat = dfeat.contiguous()
        d3 = _tc_act(n, R, C, 64, dev)
        nat.check(L.heist_train_pool_bwd(P(dfeat), P(m3), n, R, C, P(d3), st), "heist_train_pool_bwd")
        part = torch.empty(int(max(L.heist_train_conv_partial_floats(k, n, R, C) for k in (1, 2, 3))),
                           dtype=torch.float32, device=dev)
        grads = {}

        def wgrad(layer, dy, xin, co, ci, qk):
            dw = torch.empty(co, ci, 3, 3, dtype=torch.float32, device=dev)
            db = torch.empty(co, dtype=torch.float32, device=dev)
            nat.check(L.heist_train_conv_wgrad(layer, P(dy), P(xin), n, R, C, P(part), P(dw), P(db), P(q[qk:]), st),
                      "heist_train_conv_wgrad")
            grads[layer] = (dw, db)

        def dgrad(layer, w, dy, mask, ch_out, qk):
            f = _tc_frag(layer, 1, w, st)
            d = _tc_act(n, R, C, ch_out, dev)
            nat.check(L.heist_train_conv(layer, 1, P(dy), n, R, C, P(f), None, P(mask), P(d), P(q[qk:]), st),
                      "heist_train_conv")
            return d, f

        d2, f3 = dgrad(3, w3, d3, m2, 64, 6)
        wgrad(3, d3, a2, 64, 64, 8)
        d1, f2 = dgrad(2, w2, d2, m1, 32, 10)
        wgrad(2, d2, a1, 64, 32, 12)
        wgrad(1, d1, x4, 32, 3, 14)
        return None, grads[1][0], grads[1][1], grads[2][0], grads[2][1], grads[3][0], grads[3][1]


class SolverNetwork(nn.Module):  # networks.py:13-131
    def __init__(self, grid_rows: int = 20, grid_cols: int = 20, num_actions: int = 5, hidden_dim: int = 256,
                 lstm_hidden: int = 128):
        super().__init__()
        self.grid_rows = grid_rows
        self.grid_cols = grid_cols
        self.hidden_dim = hidden_dim
        self.lstm_hidden = lstm_hidden
        self.conv1 = nn.Conv2d(3, 32, kernel_size=3, padding=1)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=3, padding=1)
        self.conv3 = nn.Conv2d(64, 64, kernel_size=3, padding=1)
        self.pool = nn.AdaptiveAvgPool2d((4, 4))
        self.fc_spatial = nn.Linear(64 * 4 * 4, hidden_dim)
        self.lstm = nn.LSTM(hidden_dim, lstm_hidden, batch_first=True)
        self.policy_head = nn.Sequential(nn.Linear(lstm_hidden, 128), nn.ReLU(), nn.Linear(128, num_actions))
        self.value_head = nn.Sequential(nn.Linear(lstm_hidden, 128), nn.ReLU(), nn.Linear(128, 1))
        self._init_weights()

    def _init_weights(self):  # networks.py:68-74
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=0.01)
                nn.init.zeros_(m.bias)

    def _init_hidden(self, batch_size: int, device):
        z = torch.zeros(1, batch_size, self.lstm_hidden, device=device)
        return z, z.clone()

    #: fp32 on a HIP device: the conv stack's bias / ReLU / pool (and their backward) fused
    #: around MIOpen's bias-free convolutions (_BackboneF32); HEIST_FUSED_TRAIN=0 or False here
    #: runs the plain torch ops
    fused_tail = True

    def _fused_tail_ok(self, state: torch.Tensor) -> bool:
        import os
        return (self.fused_tail and os.environ.get("HEIST_FUSED_TRAIN", "1") != "0" and state.is_cuda
                and state.dtype == torch.float32 and state.dim() == 4 and state.shape[1] == 3
                and state.shape[2] >= 4 and state.shape[3] >= 4 and state.shape[0] > 0
                and not state.requires_grad  # _BackboneF32 forms no input gradient
                and self.conv1.weight.dtype == torch.float32
                and not torch.is_autocast_enabled("cuda") and self.conv3.out_channels == 64
                and tuple(self.pool.output_size) == (4, 4))

    #: fp32 on a HIP device at 20 x 20: every conv pass on the hand-written fp32-MFMA kernels
    #: (_BackboneMFMA32); HEIST_TRAIN_CONV=0 or False here keeps MIOpen (_BackboneF32)
    mfma_train = True

    def _train_conv_ok(self, state: torch.Tensor) -> bool:
        import os
        if not (self.mfma_train and os.environ.get("HEIST_TRAIN_CONV", "1") != "0" and self._fused_tail_ok(state)):
            return False
        from . import _native
        convs = (self.conv1, self.conv2, self.conv3)
        return (bool(_native.lib().heist_train_conv_supported(state.shape[2], state.shape[3]))
                and [(m.in_channels, m.out_channels) for m in convs] == [(3, 32), (32, 64), (64, 64)]
                and all(m.kernel_size == (3, 3) and m.padding == (1, 1) and m.stride == (1, 1) and m.dilation == (1, 1)
                        and m.groups == 1 and m.bias is not None for m in convs))

    def features(self, state: torch.Tensor) -> torch.Tensor:
        if self._train_conv_ok(state):
            x = _BackboneMFMA32.apply(state, self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias,
                                      self.conv3.weight, self.conv3.bias)
            return F.relu(_linear(x, self.fc_spatial.weight, self.fc_spatial.bias))
        if self._fused_tail_ok(state):
            x = _BackboneF32.apply(state, self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias,
                                   self.conv3.weight, self.conv3.bias)
            return F.relu(_linear(x, self.fc_spatial.weight, self.fc_spatial.bias))
        x = F.relu(self.conv1(state))
        x = F.relu(self.conv2(x))
        x = F.relu(self.conv3(x))
        x = self.pool(x)
        return F.relu(_linear(x.reshape(state.shape[0], -1), self.fc_spatial.weight, self.fc_spatial.bias))

    def lstm_step(self, x: torch.Tensor, hidden: Tuple[torch.Tensor, torch.Tensor]):
        """One LSTM time step with nn.LSTM's gate order (i, f, g, o)."""
        h, c = hidden[0][0], hidden[1][0]
        gx = _linear(x, self.lstm.weight_ih_l0, self.lstm.bias_ih_l0)
        gh = _linear(h, self.lstm.weight_hh_l0, self.lstm.bias_hh_l0)
        if (not torch.is_grad_enabled() and gx.is_cuda and gx.dtype == torch.float32 and gh.dtype == torch.float32
                and c.dtype == torch.float32):
            # inference (the rollout): the pointwise part as one HIP kernel (heist_lstm_cell),
            # the ten torch kernels' roundings in their order
            from . import _native as nat
            gx, gh, c = gx.contiguous(), gh.contiguous(), c.contiguous()
            h1, c1 = torch.empty_like(c), torch.empty_like(c)
            nat.check(nat.lib().heist_lstm_cell(nat.ptr(gx), nat.ptr(gh), nat.ptr(c), nat.ptr(h1), nat.ptr(c1),
                                                c.shape[1], c.shape[0], nat.stream(gx.device)), "heist_lstm_cell")
            return h1, (h1.unsqueeze(0), c1.unsqueeze(0))
        gates = gx + gh
        i, f, g, o = gates.chunk(4, dim=1)
        c1 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        h1 = torch.sigmoid(o) * torch.tanh(c1)
        return h1, (h1.unsqueeze(0), c1.unsqueeze(0))

    def forward(self, state: torch.Tensor, hidden: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        """(logits [B,A], value [B,1], (h, c) [1,B,H]) -- networks.py:76-116."""
        b = state.shape[0]
        spatial = self.features(state)
        if hidden is None:
            hidden = self._init_hidden(b, state.device)
        out, new_hidden = self.lstm_step(spatial, hidden)
        return _mlp_head(self.policy_head, out), _mlp_head(self.value_head, out), new_hidden

    # -- fused backbone (heist_solver_features, bf16 MFMA) -----------------------------
    def fused_supported(self, state: torch.Tensor) -> bool:
        """The HIP backbone covers 20x20, 10x10 and (row bands) 32x32 grids on a HIP device."""
        return state.is_cuda and state.dim() == 4 and tuple(state.shape[1:]) in ((3, 20, 20), (3, 10, 10), (3, 32, 32))

    def _packed_backbone(self) -> torch.Tensor:
        """conv1-3 weights in the kernel's MFMA fragment layout, re-packed (one small launch)
        whenever a conv parameter changed (optimizer steps bump the tensor versions)."""
        from . import _native
        convs = (self.conv1, self.conv2, self.conv3)
        key = tuple((m.weight.data_ptr(), m.weight._version, m.bias.data_ptr(), m.bias._version) for m in convs)
        cache = getattr(self, "_pack_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        dev = self.conv1.weight.device
        L = _native.lib()
        buf = torch.empty(L.heist_solver_packed_bytes(), dtype=torch.uint8, device=dev)
        ws = [t.detach().float().contiguous() for m in convs for t in (m.weight, m.bias)]
        _native.check(L.heist_solver_pack(*(_native.ptr(t) for t in ws), _native.ptr(buf), _native.stream(dev)),
                      "heist_solver_pack")
        self._pack_cache = (key, buf, ws)  # ws keeps the fp32 sources alive until the pack ran
        return buf

    def features_fused(self, state: torch.Tensor) -> torch.Tensor:
        """Pooled conv features [B, 1024] (networks.py:93-100) from the HIP kernel:
        bf16 operands, fp32 accumulation; inference only (no autograd)."""
        from . import _native
        if not self.fused_supported(state):
            raise _native.HeistError("fused Solver backbone needs [B,3,R,R], R in (10, 20, 32), on a HIP device")
        x = state.detach().float().contiguous()
        packed = self._packed_backbone()
        out = torch.empty(x.shape[0], 1024, dtype=torch.float32, device=x.device)
        _native.check(_native.lib().heist_solver_features(_native.ptr(x), x.shape[0], x.shape[2], x.shape[3],
                                                          _native.ptr(packed), _native.ptr(out),
                                                          _native.stream(x.device)), "heist_solver_features")
        return out

    def head_supported(self) -> bool:
        """The fused head kernel's fixed widths (networks.py:38-60 defaults)."""
        return (self.hidden_dim == 256 and self.lstm_hidden == 128 and self.policy_head[0].out_features == 128
                and self.value_head[0].out_features == 128 and 1 <= self.policy_head[2].out_features <= 7)

    def _packed_head(self) -> torch.Tensor:
        from . import _native
        mods = [self.fc_spatial.weight, self.fc_spatial.bias, self.lstm.weight_ih_l0, self.lstm.weight_hh_l0,
                self.lstm.bias_ih_l0, self.lstm.bias_hh_l0, self.policy_head[0].weight, self.policy_head[0].bias,
                self.value_head[0].weight, self.value_head[0].bias, self.policy_head[2].weight,
                self.policy_head[2].bias, self.value_head[2].weight, self.value_head[2].bias]
        key = tuple((t.data_ptr(), t._version) for t in mods)
        cache = getattr(self, "_head_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        dev = self.fc_spatial.weight.device
        L = _native.lib()
        buf = torch.empty(L.heist_solver_head_packed_bytes(), dtype=torch.uint8, device=dev)
        ws = [t.detach().float().contiguous() for t in mods]
        _native.check(L.heist_solver_head_pack(*(_native.ptr(t) for t in ws), self.policy_head[2].out_features,
                                               _native.ptr(buf), _native.stream(dev)), "heist_solver_head_pack")
        self._head_cache = (key, buf, ws)
        return buf

    @torch.no_grad()
    def act_fused(self, state: torch.Tensor, hidden: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                  seed: int = 0, counter: int = 0, want_logits: bool = False):
        """get_action (networks.py:124-131) for a batch, entirely on the fused kernels:
        backbone (heist_solver_features) + head (heist_solver_head: fc, LSTM cell, heads,
        Categorical sample).  Returns (action [B] int64, log_prob [B], value [B],
        (h, c) [1,B,128], logits [B,A] or None)."""
        from . import _native
        b = state.shape[0]
        feat = self.features_fused(state)
        dev = feat.device
        A = self.policy_head[2].out_features
        packed = self._packed_head()
        h_in = c_in = None
        if hidden is not None:
            h_in = hidden[0].reshape(b, self.lstm_hidden).float().contiguous()
            c_in = hidden[1].reshape(b, self.lstm_hidden).float().contiguous()
        h1 = torch.empty(1, b, self.lstm_hidden, device=dev)
        c1 = torch.empty(1, b, self.lstm_hidden, device=dev)
        value = torch.empty(b, device=dev)
        action = torch.empty(b, dtype=torch.int64, device=dev)
        logp = torch.empty(b, device=dev)
        logits = torch.empty(b, A, device=dev) if want_logits else None
        _native.check(_native.lib().heist_solver_head(
            _native.ptr(feat), _native.ptr(h_in), _native.ptr(c_in), b, _native.ptr(packed), A,
            seed & 0xFFFFFFFFFFFFFFFF, counter & 0xFFFFFFFFFFFFFFFF, _native.ptr(logits), _native.ptr(value),
            _native.ptr(action), _native.ptr(logp), _native.ptr(h1), _native.ptr(c1), _native.stream(dev)),
            "heist_solver_head")
        return action, logp, value, (h1, c1), logits

    @torch.no_grad()
    def forward_fused(self, state: torch.Tensor, hidden: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        """forward() with the conv backbone on the fused HIP kernel (rollout inference)."""
        b = state.shape[0]
        spatial = F.relu(self.fc_spatial(self.features_fused(state)))
        if hidden is None:
            hidden = self._init_hidden(b, state.device)
        out, new_hidden = self.lstm_step(spatial, hidden)
        return self.policy_head(out), self.value_head(out), new_hidden

    def get_action(self, state: torch.Tensor, hidden=None):  # networks.py:124-131
        logits, value, new_hidden = self.forward(state, hidden)
        dist = torch.distributions.Categorical(F.softmax(logits, dim=-1))
        action = dist.sample()
        return action, dist.log_prob(action), value, new_hidden


class ArchitectNetwork(nn.Module):  # networks.py:134-335
    def __init__(self, grid_rows: int = 20, grid_cols: int = 20, num_asset_types: int = 3, hidden_dim: int = 256):
        super().__init__()
        self.grid_rows = grid_rows
        self.grid_cols = grid_cols
        self.num_asset_types = num_asset_types
        self.encoder = nn.Sequential(
            nn.Conv2d(1, 32, kernel_size=3, padding=1), nn.ReLU(),
            nn.Conv2d(32, 64, kernel_size=3, padding=1), nn.ReLU(),
            nn.Conv2d(64, 64, kernel_size=3, padding=1), nn.ReLU())
        self.global_pool = nn.AdaptiveAvgPool2d((4, 4))
        self.fc_global = nn.Linear(64 * 4 * 4, hidden_dim)
        self.decoder = nn.Sequential(
            nn.Conv2d(64, 64, kernel_size=3, padding=1), nn.ReLU(),
            nn.Conv2d(64, 32, kernel_size=3, padding=1), nn.ReLU(),
            nn.Conv2d(32, num_asset_types + 1, kernel_size=1))
        self.value_head = nn.Sequential(nn.Linear(hidden_dim, 128), nn.ReLU(), nn.Linear(128, 1))
        self.camera_fov_head = nn.Linear(hidden_dim, 1)
        self.camera_speed_head = nn.Linear(hidden_dim, 1)
        self.camera_heading_head = nn.Linear(hidden_dim, 1)
        self._init_weights()

    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.Linear):
                nn.init.orthogonal_(m.weight, gain=0.01)
                nn.init.zeros_(m.bias)

    def forward(self, grid_state: torch.Tensor):  # networks.py:205-239
        features = self.encoder(grid_state)
        g = self.global_pool(features).reshape(features.shape[0], -1)
        g = F.relu(self.fc_global(g))
        placement_logits = self.decoder(features)
        state_value = self.value_head(g)
        camera_params = {
            "fov": torch.sigmoid(self.camera_fov_head(g)) * 90 + 30,
            "speed": torch.sigmoid(self.camera_speed_head(g)) * 30 + 5,
            "heading": torch.sigmoid(self.camera_heading_head(g)) * 360,
        }
        return placement_logits, state_value, camera_params

    def value(self, grid_state: torch.Tensor) -> torch.Tensor:
        """state_value of forward() alone (encoder -> pool -> fc_global -> value_head): the only
        output the Architect update's loss depends on (its policy term carries no gradient), so
        the gradients equal those of the full forward (the decoder and camera heads get none)."""
        features = self.encoder(grid_state)
        g = self.global_pool(features).reshape(features.shape[0], -1)
        return self.value_head(F.relu(self.fc_global(g)))

    @staticmethod
    def _generate_patrol(row: int, col: int, grid_h: int, grid_w: int) -> list:  # networks.py:324-335
        offsets = [(0, 0), (0, 1), (0, 2), (1, 2), (2, 2), (2, 1), (2, 0), (1, 0)]
        return [(max(1, min(grid_h - 2, row + dr - 1)), max(1, min(grid_w - 2, col + dc - 1))) for dr, dc in offsets]

    def sample_assets(self, grid_state: torch.Tensor, n: int, temperature: float = 1.0,
                      generator: Optional[torch.Generator] = None):
        """Forward once, then draw n per-cell asset maps from softmax(logits / T).

        Returns (asset_map [n,R,C] int64, total_log_prob [n], value [1,1], cam_params dict).
        total_log_prob follows Categorical(probs).log_prob summed over all cells
        (networks.py:269-271, :320)."""
        logits, value, cam = self.forward(grid_state)
        probs = F.softmax(logits / temperature, dim=1)  # [1,4,R,C]
        _, k, h, w = probs.shape
        flat = probs[0].reshape(k, h * w).t()  # [RC,4]
        pn = flat / flat.sum(-1, keepdim=True)
        samples = torch.multinomial(pn.repeat(n, 1), 1, replacement=True, generator=generator).reshape(n, h * w)
        eps = torch.finfo(pn.dtype).eps
        logp = torch.log(pn.clamp(eps, 1 - eps))  # probs_to_logits
        total = logp.gather(1, samples.t()).sum(0)  # [n]
        return samples.reshape(n, h, w), total, value, cam

    def generate_layout(self, grid_state: torch.Tensor, budget: int, temperature: float = 1.0):
        """networks.py:241-322 for one layout: (walls, cameras, guards, total_log_prob, value)."""
        from .architect_decode import decode_layouts
        amap, total, value, cam = self.sample_assets(grid_state, 1, temperature)
        lay = decode_layouts(amap, cam, budget)
        walls, cams, guards = lay.to_lists()[0]
        return walls, cams, guards, total[0], value
