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

import torch
import torch.nn as nn
import torch.nn.functional as F


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

    def features(self, state: torch.Tensor) -> torch.Tensor:
        x = F.relu(self.conv1(state))
        x = F.relu(self.conv2(x))
        x = F.relu(self.conv3(x))
        x = self.pool(x)
        return F.relu(self.fc_spatial(x.reshape(state.shape[0], -1)))

    def lstm_step(self, x: torch.Tensor, hidden: Tuple[torch.Tensor, torch.Tensor]):
        """One LSTM time step with nn.LSTM's gate order (i, f, g, o)."""
        h, c = hidden[0][0], hidden[1][0]
        gates = F.linear(x, self.lstm.weight_ih_l0, self.lstm.bias_ih_l0) + \
            F.linear(h, self.lstm.weight_hh_l0, self.lstm.bias_hh_l0)
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
        return self.policy_head(out), self.value_head(out), new_hidden

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
