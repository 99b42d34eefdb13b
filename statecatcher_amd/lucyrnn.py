"""Drop-in of the reference's native LucyRNN (/root/reference/lucyrnn.py) on the HIP scans.

Same classes, constructor, parameter names (``layers.{l}.input_proj``, ``layernorm_{in,r,z,h}``,
``W_fused`` or ``W_{r,z,k,v,h,decay}``, ``output_proj``), ``forward(x, hidden_states=None,
masks=None)`` and return values as lucyrnn.py:8-191, with the reference's train/infer
semantics reproduced exactly (in train mode the decay scan starts from 0, its
output is fed to the cell as s_prev so the decay step is applied twice, and s is never
carried; infer mode is the true recurrence).

The reference runs Python loops over time (lucyrnn.py:155-166, :174-182).  Here every layer is
evaluated for all T at once: its gates depend only on the layer input, and both recurrences are
first-order LINEAR scans:
    s_t = dec_t s_{t-1} + k_t v_t                     (sc_decay_scan, initial state s_prev)
    h_t = z_t h_{t-1} + (1 - z_t) c_t                 (sc_decay_scan with decay = z)
and a frame mask m turns either into  x_t = (m z_t + 1 - m) x_{t-1} + m (...)  — still linear.
Both scans run on the HIP decay-scan kernel (decay_scan.hip) in fp32 with autograd; the
projections and LayerNorms are GEMMs / torch ops around them.

Masks: the reference's ``masks[:, t, :].unsqueeze(-1)`` broadcasts a [B,1,1] mask against [B,D]
states (lucyrnn.py:164, :176), which only works without masks; here masks of shape [B,T] or
[B,T,1] blend per (b, t) as lucyrnn.py:66-68 intends.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .lucyrnn_conf import LucyRNNConfig
from .ops import decay_scan


class LucyRNNCell(nn.Module):
    """lucyrnn.py:8-70.  forward() is the single-step cell (streaming inference)."""

    def __init__(self, input_dim, hidden_dim, fused_ops=False, layer_norm=True):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.fused_ops = fused_ops
        self.layer_norm = layer_norm
        self.input_proj = nn.Linear(input_dim, hidden_dim)
        self.layernorm_in = nn.LayerNorm(hidden_dim) if layer_norm else nn.Identity()
        self.layernorm_r = nn.LayerNorm(hidden_dim) if layer_norm else nn.Identity()
        self.layernorm_z = nn.LayerNorm(hidden_dim) if layer_norm else nn.Identity()
        self.layernorm_h = nn.LayerNorm(hidden_dim) if layer_norm else nn.Identity()
        if fused_ops:
            self.W_fused = nn.Linear(hidden_dim, 6 * hidden_dim)
        else:
            self.W_r = nn.Linear(hidden_dim, hidden_dim)
            self.W_z = nn.Linear(hidden_dim, hidden_dim)
            self.W_k = nn.Linear(hidden_dim, hidden_dim)
            self.W_v = nn.Linear(hidden_dim, hidden_dim)
            self.W_h = nn.Linear(hidden_dim, hidden_dim)
            self.W_decay = nn.Linear(hidden_dim, hidden_dim)
        self.init_weights()

    def init_weights(self):
        """lucyrnn.py:34-42: orthogonal weight matrices, unit/zero LayerNorms."""
        for name, param in self.named_parameters():
            if "weight" in name and param.dim() > 1:
                nn.init.orthogonal_(param)
        if self.layer_norm:
            for ln in [self.layernorm_in, self.layernorm_r, self.layernorm_z, self.layernorm_h]:
                nn.init.constant_(ln.bias, 0)
                nn.init.constant_(ln.weight, 1.0)

    def gates(self, x):
        """u and the per-step terms that depend only on the input: (u, z, k, v, h_pre, dec)
        with h_pre None in the unfused form (its W_h sees u + s)."""
        u = self.layernorm_in(self.input_proj(x))
        if self.fused_ops:
            _, z, k, v, h_pre, dl = self.W_fused(u).chunk(6, dim=-1)
            z = torch.sigmoid(self.layernorm_z(z))
        else:
            z = torch.sigmoid(self.layernorm_z(self.W_z(u)))
            k, v, dl, h_pre = self.W_k(u), self.W_v(u), self.W_decay(u), None
        return u, z, k, v, h_pre, torch.sigmoid(dl)

    def candidate(self, u, h_pre, s):
        """c = tanh(LN_h(h_pre + s)) (fused, :54) or tanh(LN_h(W_h(u + s))) (unfused, :62)."""
        if self.fused_ops:
            return torch.tanh(self.layernorm_h(h_pre + s))
        return torch.tanh(self.layernorm_h(self.W_h(u + s)))

    def forward(self, x, h_prev, s_prev, mask=None):
        u, z, k, v, h_pre, dec = self.gates(x)
        s = dec * s_prev + k * v
        c = self.candidate(u, h_pre, s)
        h = (1 - z) * c + z * h_prev
        if mask is not None:
            h = mask * h + (1 - mask) * h_prev
            s = mask * s + (1 - mask) * s_prev
        return h, s


def _masked(decay, drive, m):
    """x_t = decay x_{t-1} + drive, blended with x_{t-1} where m = 0."""
    if m is None:
        return decay, drive
    return m * decay + (1 - m), m * drive


def _scan(drive, decay, init):
    # fp32 state; the HIP kernel carries the autograd of kv, decay and init
    return decay_scan(drive.float(), decay.float(), None if init is None else init.float())


class LucyRNN(nn.Module):
    """lucyrnn.py:72-191 with every layer evaluated over the whole segment."""

    def __init__(self, config: LucyRNNConfig):
        super().__init__()
        self.config = config
        if config.kernel_impl not in ["native", "triton"]:
            raise ValueError("kernel_impl must be either 'native' or 'triton'")
        self.layers = nn.ModuleList()
        for i in range(config.num_layers):
            d_in = config.input_dim * config.stack_order if i == 0 else config.hidden_dim
            self.layers.append(LucyRNNCell(d_in, config.hidden_dim, config.fused_ops,
                                           config.layer_norm))
        self.output_proj = nn.Linear(config.hidden_dim, config.vocab_size)
        nn.init.zeros_(self.output_proj.weight)
        nn.init.zeros_(self.output_proj.bias)

    def _stack(self, x, masks):
        B, T, Fd = x.shape
        k = self.config.stack_order
        if k > 1:
            Tt = T - T % k
            x = x[:, :Tt].reshape(B, Tt // k, Fd * k)
            if masks is not None:
                masks = masks[:, :Tt].reshape(B, Tt // k, k).all(dim=-1)
        if masks is not None:
            masks = masks.reshape(masks.shape[0], masks.shape[1], 1).to(torch.float32)
        return x, masks

    def forward(self, x, hidden_states=None, masks=None):
        cfg = self.config
        x, m = self._stack(x, masks)
        B, T, _ = x.shape
        D = cfg.hidden_dim
        if hidden_states is None:
            h = [torch.zeros(B, D, device=x.device) for _ in range(cfg.num_layers)]
            s = [torch.zeros(B, D, device=x.device) for _ in range(cfg.num_layers)]
        else:
            h, s = hidden_states
            h, s = list(h), list(s)
        inp = x
        for l, layer in enumerate(self.layers):
            u, z, k, v, h_pre, dec = layer.gates(inp)
            kv = k * v
            if cfg.is_training:
                # lucyrnn.py:109-168: scan from 0, then the cell re-applies the step to the
                # scan state (s_prev = s_all[t]); s is not carried (F9)
                if cfg.decay_mode == "learned":
                    s_all = _scan(kv, dec, None)
                elif cfg.decay_mode == "prefix_sum":
                    tt = torch.arange(T, device=x.device, dtype=torch.float32)
                    log_w = torch.cumsum(torch.log(torch.exp(-cfg.lambda_decay * tt) + 1e-7), 0)
                    log_w = log_w.view(1, T, 1)
                    s_all = torch.cumsum(kv * torch.exp(log_w), dim=1) / (torch.exp(log_w) + 1e-7)
                else:
                    raise ValueError(f"Unknown decay_mode: {cfg.decay_mode}")
                s_cell = dec * s_all + kv
            else:
                # lucyrnn.py:172-184: the true recurrence, s carried across segments
                d_s, k_s = _masked(dec, kv, m)
                s_cell = _scan(k_s, d_s, s[l])
                s[l] = s_cell[:, -1]
            c = layer.candidate(u, h_pre, s_cell)
            d_h, k_h = _masked(z, (1 - z) * c, m)
            h_all = _scan(k_h, d_h, h[l])
            h[l] = h_all[:, -1]
            inp = h_all
        logits = self.output_proj(inp)
        if cfg.return_last_states:
            return logits, (h, s)
        return logits

    @torch.no_grad()
    def step(self, x_t, states):
        """One streaming frame through all layers (lucyrnn.py:174-182 body): x_t [B, F*stack],
        states (h list, s list) -> (logits [B, V], states)."""
        h, s = list(states[0]), list(states[1])
        inp = x_t
        for l, layer in enumerate(self.layers):
            h[l], s[l] = layer(inp, h[l], s[l])
            inp = h[l]
        return self.output_proj(inp), (h, s)
