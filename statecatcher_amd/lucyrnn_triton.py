"""Drop-in replacement of the reference's lucyrnn_triton.py module API on MI355X.

Same classes, constructor arguments, forward signatures, state nesting and state_dict keys as
/root/reference/lucyrnn_triton.py:8-155 (`LinearSafe`, `LucyRNNCellTriton`, `LucyRNNtriton`),
so model.py / train.py can import it unchanged.  The Triton kernel launch
(lucyrnn_triton.py:61-73) is replaced by the HIP scan (statecatcher_amd/csrc/lucy_scan.hip via
ops.LucyScanFn), which also has a backward.

Differences from the reference, all deliberate:
  * gradients flow into the recurrent layers (the reference's outputs have no grad_fn, F2);
  * h0 is read through .contiguous(), so the carried out[:, -1] view is honoured (F3);
  * bf16 / fp16 gates (e.g. under torch.autocast) run; state arithmetic stays fp32 (F4);
  * s_last and the carried h (out[:, -1]) are returned in fp32 whatever the gate dtype, so a
    bf16-autocast run carries its state across segments unrounded, as the fp32 reference does.
"""
import threading

import torch
import torch.nn as nn

from .lucyrnn_conf import LucyRNNConfig
from .ops import (LN_FOLD_MODE, cell_image_spec, colsum, fold_images, layer_norm,
                  layer_norm_supported, ln_fold_ok,
                  lucy_cell, lucy_cell_ln, proj_dgrad, weight_images, wgrad_splitk)


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b in the autocast dtype; backward with a split-K weight gradient.  imgs:
    (W, W^T, b) bf16 images from ops.weight_images, or None (cast here)."""

    @staticmethod
    def forward(ctx, x, w, b, cdtype, imgs=None):
        xc = x.to(cdtype)
        if imgs is not None:
            wc, wt, bc = imgs
        else:
            wc, wt = w.to(cdtype), None
            bc = b.to(cdtype) if b is not None else None
        out = torch.addmm(bc, xc, wc.t()) if b is not None else xc @ wc.t()
        ctx.save_for_backward(xc, wc if wt is None else None, wt)
        ctx.meta = (x.dtype, w.dtype, b is not None, cdtype)
        return out

    @staticmethod
    def backward(ctx, dy):
        xc, wc, wt = ctx.saved_tensors
        xdt, wdt, has_b, cdt = ctx.meta
        dy = dy.to(cdt)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (torch.matmul(dy, wt.t()) if wt is not None else proj_dgrad(dy, wc)).to(xdt)
        dw = wgrad_splitk(dy, xc).to(wdt) if ctx.needs_input_grad[1] else None
        db = colsum(dy).to(wdt) if has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None


# compute_loss's request to hand the output projection to the loss (ops.CTCHeadFn): set, the next
# LucyRNNtriton forward on this thread that can fuse stores (hidden, output_proj, images, the
# last scan's split-precision buffer or None) here and returns DEFERRED_LOGITS for the logits
_HEAD = threading.local()
DEFERRED_LOGITS = object()


class defer_output_head:
    """with defer_output_head() as h: ... model(...) ...; h.taken is (x, output_proj, images,
    wide) when the encoder deferred its output projection, else None."""

    def __enter__(self):
        self.taken = None
        _HEAD.req = self
        return self

    def __exit__(self, *exc):
        _HEAD.req = None
        return False


class LinearSafe(nn.Module):
    """y = x W^T + b over the flattened leading dims (lucyrnn_triton.py:8-25)."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.weight)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x, imgs=None):
        x_flat = x.reshape(-1, x.shape[-1])
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            cdt = torch.get_autocast_dtype("cuda")
        else:
            cdt = torch.promote_types(x.dtype, self.weight.dtype)
        if imgs is not None and cdt != torch.bfloat16:
            imgs = None
        with torch.autocast("cuda", enabled=False):
            # one GEMM with the bias in its epilogue (hipBLASLt); the reference adds it after
            out = _LinearFn.apply(x_flat, self.weight, self.bias, cdt, imgs)
        return out.view(*x.shape[:-1], self.weight.shape[0])

    def image_specs(self, needs_dx):
        """weight_images specs for a bf16 forward: W (+ W^T for the input gradient), b."""
        w, b = self.weight, self.bias
        if not (w.is_cuda and w.dtype == torch.float32 and w.stride(1) == 1
                and (b is None or (b.dtype == torch.float32 and b.stride(0) == 1))):
            return None
        specs = [(w, 0, w.shape[1], needs_dx)]
        if b is not None:
            specs.append((b, 0, b.shape[0], False))
        return specs


class LayerNormHip(nn.LayerNorm):
    """nn.LayerNorm (same parameters / state_dict) whose forward runs layernorm.hip in the
    activation's own dtype: under autocast the bf16 scan output is normalised straight into the
    bf16 input of the next gate GEMM, with fp32 statistics."""

    def forward(self, x):
        if x.is_cuda and self.elementwise_affine and len(self.normalized_shape) == 1 \
                and layer_norm_supported(x):
            with torch.autocast("cuda", enabled=False):
                return layer_norm(x, self.weight, self.bias, self.eps)
        return super().forward(x)


class LucyRNNCellTriton(nn.Module):
    """7-gate projection + HIP scan (lucyrnn_triton.py:27-75)."""

    def __init__(self, input_dim, hidden_dim):
        super().__init__()
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.linear = LinearSafe(input_dim, 7 * hidden_dim)
        self._init_weights()

    def _init_weights(self):
        nn.init.xavier_uniform_(self.linear.weight)
        if self.linear.bias is not None:
            D = self.hidden_dim
            with torch.no_grad():   # gate-aware bias init, lucyrnn_triton.py:41-48
                self.linear.bias[0 * D:1 * D].zero_()      # r
                self.linear.bias[1 * D:2 * D].fill_(1.0)   # z
                self.linear.bias[2 * D:3 * D].zero_()      # k
                self.linear.bias[3 * D:4 * D].zero_()      # v
                self.linear.bias[4 * D:5 * D].zero_()      # h_pre
                self.linear.bias[5 * D:6 * D].fill_(2.0)   # decay
                self.linear.bias[6 * D:7 * D].fill_(0.5)   # alpha

    def forward(self, x, h0, s0):
        """(out [B,T,D], s_out [B,D]) as lucyrnn_triton.py:50-75 returns them."""
        out, s_out, _ = self.forward_with_h(x, h0, s0)
        return out, s_out

    def forward_with_h(self, x, h0, s0, imgs=None, split_sink=None, rec_sink=None):
        """(out, s_out, h_last): h_last = out[:, -1] in fp32, unrounded by a 16-bit out (the
        state LucyRNNtriton carries).  Projection GEMM + scan are one autograd node: the scan
        backward hands the bias gradient back from registers, the weight gradient runs on the
        MFMA split-L kernel.  imgs: this layer's entry of ops.weight_images (bf16 only);
        split_sink: ops.LucyCellFn's (the scan's split-precision output planes); rec_sink: its
        LayerNorm block records for a folded next layer."""
        w, b = self.linear.weight, self.linear.bias
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            cdt = torch.get_autocast_dtype("cuda")
        else:
            cdt = torch.promote_types(x.dtype, w.dtype)
        if b is None:
            b = torch.zeros(w.shape[0], dtype=w.dtype, device=w.device)
        if imgs is not None and cdt != torch.bfloat16:
            imgs = None
        with torch.autocast("cuda", enabled=False):
            return lucy_cell(x, w, b, h0, s0, cdt, imgs, split_sink, rec_sink)


class LucyRNNtriton(nn.Module):
    """L-layer LucyRNN stack with inter-layer LayerNorm and a vocab projection
    (lucyrnn_triton.py:77-155).  forward(x, hidden_states=None, masks=None) ->
    (logits, (final_h, final_s)) with final_h/final_s nested [track][layer] of [B, D]."""

    def __init__(self, config: LucyRNNConfig):
        super().__init__()
        assert config.fused_ops
        assert not config.layer_norm
        assert config.stack_order == 1
        assert config.decay_mode == 'learned'

        self.config = config
        self.num_tracks = getattr(config, "num_tracks", 1)

        self.tracks = nn.ModuleList()
        self.norms = nn.ModuleList()
        for _ in range(self.num_tracks):
            layers = nn.ModuleList()
            norms = nn.ModuleList()
            for i in range(config.num_layers):
                input_dim = config.input_dim if i == 0 else config.hidden_dim
                layers.append(LucyRNNCellTriton(input_dim, config.hidden_dim))
                if i < config.num_layers - 1:
                    norms.append(LayerNormHip(config.hidden_dim))
            self.tracks.append(layers)
            self.norms.append(norms)

        self.merge_proj = (nn.Identity() if self.num_tracks == 1 else
                           LinearSafe(config.hidden_dim * self.num_tracks, config.hidden_dim))
        self.output_proj = LinearSafe(config.hidden_dim, config.vocab_size)
        nn.init.zeros_(self.output_proj.weight)
        nn.init.zeros_(self.output_proj.bias)

    def forward(self, x, hidden_states=None, masks=None):
        B, T, _ = x.shape
        L = self.config.num_layers
        H = self.config.hidden_dim
        if hidden_states is None:   # lucyrnn_triton.py:119-120, one zero-fill for all states
            z = torch.zeros(2, self.num_tracks, L, B, H, device=x.device, dtype=x.dtype)
            h = [[z[0, k, l] for l in range(L)] for k in range(self.num_tracks)]
            s = [[z[1, k, l] for l in range(L)] for k in range(self.num_tracks)]
        else:
            h, s = hidden_states

        cell_imgs, out_imgs, fold = self._weight_images(x)
        req = getattr(_HEAD, "req", None)
        op = self.output_proj
        if req is not None and not (out_imgs is not None and out_imgs[1] is not None
                                    and self.num_tracks == 1 and op.bias is not None
                                    and op.weight.dtype == torch.float32
                                    and op.bias.dtype == torch.float32
                                    and self.config.hidden_dim % 4 == 0):
            # CTCHeadFn's preconditions (ops.ctc_head_supported; sc_ctc_split_rows reads the
            # weight rows in 4-element pieces): otherwise the projection runs here, unfused
            req = None
        sink = [] if req is not None else None
        track_outputs, final_h, final_s = [], [], []
        for t in range(self.num_tracks):
            x_t = x
            h_t, s_t = h[t], s[t]
            layers = self.tracks[t]
            norms = self.norms[t]
            rec = None
            for l, layer in enumerate(layers):
                last = l == len(layers) - 1
                # h carry = out[:, -1] (lucyrnn_triton.py:135), taken in fp32 from the scan and
                # contiguous
                # (block records for the next layer: the scan-side fold only)
                rsink = [] if fold and not last and LN_FOLD_MODE == 1 else None
                if fold and l > 0:
                    # norms[l-1] folded into this layer's projection (ops.LucyCellLNFn): x_t is
                    # the previous layer's raw output, rec its block records
                    ln = norms[l - 1]
                    x_t, s_t[l], h_t[l] = lucy_cell_ln(
                        x_t, layer.linear.weight, layer.linear.bias, ln.weight, ln.bias, h_t[l],
                        s_t[l], fold[(t, l)], rec, ln.eps, sink if last else None, rsink)
                else:
                    x_t, s_t[l], h_t[l] = layer.forward_with_h(
                        x_t, h_t[l], s_t[l], cell_imgs.get((t, l)) if cell_imgs else None,
                        sink if last else None, rsink)
                rec = rsink[0] if rsink else None
                if l < len(norms) and not fold:
                    x_t = norms[l](x_t)
            track_outputs.append(x_t)
            final_h.append(h_t)
            final_s.append(s_t)

        if self.num_tracks == 1:
            x = track_outputs[0]
        else:
            x = self.merge_proj(torch.cat(track_outputs, dim=-1))
        if req is not None:
            # the last layer's scan wrote [x_hi | x_hi | x_lo] (sink) when its gates were bf16
            req.taken = (x, self.output_proj, out_imgs, sink[0] if sink else None)
            _HEAD.req = None
            logits = DEFERRED_LOGITS
        else:
            logits = self.output_proj(x.contiguous(), out_imgs)
        if self.config.return_last_states:
            return logits, (final_h, final_s)
        return logits

    def _fold_ok(self):
        """Every layer after the first takes its LayerNorm folded into its projection
        (ops.LucyCellLNFn): D of 512 / 1024, affine LayerNorms, biased fp32 projections."""
        if not ln_fold_ok(self.config.hidden_dim) or self.config.num_layers < 2:
            return False
        for layers, norms in zip(self.tracks, self.norms):
            for l, layer in enumerate(layers):
                w, b = layer.linear.weight, layer.linear.bias
                if b is None or w.dtype != torch.float32 or not w.is_cuda or w.stride(1) != 1:
                    return False
            for ln in norms:
                if not (ln.elementwise_affine and ln.weight is not None and ln.bias is not None
                        and ln.weight.dtype == torch.float32 and ln.weight.is_contiguous()
                        and ln.bias.is_contiguous()):
                    return False
        return True

    def _weight_images(self, x):
        """bf16 images of every projection weight for this forward (ops.weight_images: one
        launch after each optimizer step, cached otherwise) when the step runs under bf16
        autocast on the GPU; ({(track, layer): (W image, W^T image)}, output-projection
        (W, W^T, b) images, {(track, layer): folded-LayerNorm images (ops.fold_images)} for layers
        1.. or None) or (None, None, None)."""
        if not (x.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return None, None, None
        grad = torch.is_grad_enabled()
        fold = self._fold_ok()
        specs, where, fspecs, fwhere = [], [], [], []
        for t, layers in enumerate(self.tracks):
            for l, layer in enumerate(layers):
                sp = cell_image_spec(layer.linear.weight, torch.bfloat16,
                                     grad and (l > 0 or x.requires_grad))
                if fold and l > 0 and sp is not None:
                    ln = self.norms[t][l - 1]
                    w, bd, kp, want_t = sp
                    fspecs.append((w, layer.linear.bias, ln.weight, ln.bias, bd, kp, want_t))
                    fwhere.append((t, l))
                elif sp is not None and layer.linear.bias is not None:
                    specs.append(sp)
                    where.append((t, l))
        if fold and len(fwhere) != sum(len(layers) - 1 for layers in self.tracks):
            return self._weight_images_plain(x, grad)   # (a layer without an image spec: no fold)
        osp = self.output_proj.image_specs(grad) if self.num_tracks == 1 else None
        imgs = weight_images(specs + (osp or []))
        cell = {w: im for w, im in zip(where, imgs)}
        out = None
        if osp:
            (wc, wt), rest = imgs[len(specs)], imgs[len(specs) + 1:]
            out = (wc, wt, rest[0][0] if rest else None)
        folded = {w: im for w, im in zip(fwhere, fold_images(fspecs))} if fold else None
        return cell, out, folded

    def _weight_images_plain(self, x, grad):
        specs, where = [], []
        for t, layers in enumerate(self.tracks):
            for l, layer in enumerate(layers):
                sp = cell_image_spec(layer.linear.weight, torch.bfloat16,
                                     grad and (l > 0 or x.requires_grad))
                if sp is not None and layer.linear.bias is not None:
                    specs.append(sp)
                    where.append((t, l))
        osp = self.output_proj.image_specs(grad) if self.num_tracks == 1 else None
        imgs = weight_images(specs + (osp or []))
        cell = {w: im for w, im in zip(where, imgs)}
        out = None
        if osp:
            (wc, wt), rest = imgs[len(specs)], imgs[len(specs) + 1:]
            out = (wc, wt, rest[0][0] if rest else None)
        return cell, out, None
