"""Streaming (frame-synchronous) decode of a native LucyRNN with fused greedy CTC — SURVEY §8(f)
row 2.

The reference's streaming path is the infer-mode loop of lucyrnn.py:172-184: for every frame,
every layer runs ``LucyRNNCell.forward`` (lucyrnn.py:44-70) on the previous layer's h, then
``output_proj`` (:186), and decoding is decoder.py:3-30 (argmax, collapse repeats, drop blanks)
over the finished sequence.  Here a frame is:

    per layer:  a = input_proj(x)             library GEMM (hipBLASLt)
                u = LayerNorm_in(a)           sc_lucy_step_ln      (csrc/lucy_step.hip)
                g = gate projection(u)        library GEMM; fused: W_fused minus the dead r rows
                h, s <- cell(g, h, s)         sc_lucy_step_cell    (+ W_h GEMM + a second cell
                                                                    stage when fused_ops=False)
    logits = output_proj(h_L)                 library GEMM
    emit   = greedy step(logits, prev)        sc_ctc_greedy_step   (csrc/decode.hip)

with h, s resident on the GPU in fp32 between calls and every buffer static, so one block of
``frames_per_call`` frames is captured once as a hipGraph (torch.cuda.CUDAGraph) and replayed:
one host launch per block instead of ~(4-6 L + 2) kernel launches per frame.

schedule="wavefront" (the default with the frame engine) runs a block of K frames as K + L - 1
stages over (frame, layer), each stage one launch per kernel kind for all its layers
(_block_wavefront): 4 (K + L - 1) + 2 launches per block instead of K (4 L + 2), identical
arithmetic.

engine="frame" (the default where it applies: hidden_dim a multiple of 16) replaces the library
GEMMs and the LayerNorm / cell kernels by the fused chain of csrc/lucy_frame.hip: per layer
    a = x W_in^T + b_in (+ row statistics)            lucy_frame_gemm
    gates on LN_in(a), cell stage in the epilogue     lucy_frame_gemm  (s, z, y / hp, statistics)
    hp = y W_h^T + b_h (+ statistics)  [unfused]      lucy_frame_gemm
    h = (1 - z~) tanh(LN_h hp) + z~ h                 lucy_frame_cellb
then logits (lucy_frame_gemm) and the greedy step: 3-4 launches per layer instead of 5-6, no
LayerNorm launch (statistics ride with the producing GEMM), MFMA on fp32 (exact f32) or bf16
weights, fp32 activations.

The decode is incremental: ``prev`` holds each stream's last argmax (-1 at stream start, as
decoder.py's ``prev_token = None``), and emit[b, t] is the token decoder.py would append at
frame t, or -1.  Frames with mask 0 (past a stream's end) keep state (lucyrnn.py:66-68) and
emit nothing.
"""
import torch

from . import ops
from .lucyrnn import LucyRNN


def _ln_params(mod, on):
    return (mod.weight.detach().float().contiguous(), mod.bias.detach().float().contiguous()) \
        if on else None


class StreamingLucyRNN:
    """Decode ``batch`` concurrent streams through ``model`` (a native LucyRNN; its weights are
    snapshotted at construction) ``frames_per_call`` model frames per call.

    dtype: activation/weight dtype of the GEMMs (fp32 = the reference's arithmetic; bf16 for
    throughput); state is fp32 either way.  graph: capture the block as a hipGraph.
    """

    def __init__(self, model: LucyRNN, batch: int, frames_per_call: int = 1,
                 dtype=torch.float32, blank: int = 0, graph: bool = True, engine: str = "auto",
                 schedule: str = "wavefront"):
        cfg = model.config
        dev = next(model.parameters()).device
        ops._lib.require_device(next(model.parameters()))
        self.cfg, self.B, self.K, self.dtype, self.blank = cfg, batch, frames_per_call, dtype, blank
        self.L, self.D, self.V = cfg.num_layers, cfg.hidden_dim, cfg.vocab_size
        self.Din = cfg.input_dim * cfg.stack_order
        D, B, K = self.D, batch, frames_per_call
        if not ops._lib.load().sc_lucy_step_supported(ops.dtype_code(torch.empty(0, dtype=dtype)), D):
            raise ValueError(f"streaming step: hidden_dim {D} / dtype {dtype} unsupported")
        w = lambda t: t.detach().to(dtype).contiguous()   # noqa: E731
        ln = cfg.layer_norm
        self.layers = []
        for cell in model.layers:
            e = {"w_in": w(cell.input_proj.weight), "b_in": w(cell.input_proj.bias),
                 "ln_in": _ln_params(cell.layernorm_in, ln), "lnz": _ln_params(cell.layernorm_z, ln),
                 "lnh": _ln_params(cell.layernorm_h, ln)}
            if cfg.fused_ops:
                # rows [0, D) are r: sigmoid(LN_r(r)) is computed by the reference and never used
                e["w_g"], e["b_g"] = w(cell.W_fused.weight[D:]), w(cell.W_fused.bias[D:])
            else:
                mods = (cell.W_z, cell.W_k, cell.W_v, cell.W_decay)
                e["w_g"] = w(torch.cat([m.weight for m in mods]))
                e["b_g"] = w(torch.cat([m.bias for m in mods]))
                e["w_h"], e["b_h"] = w(cell.W_h.weight), w(cell.W_h.bias)
            self.layers.append(e)
        self.w_out, self.b_out = w(model.output_proj.weight), w(model.output_proj.bias)
        # sc_lucy_frame_gemm keeps a workgroup's A rows in LDS: K <= 2048 (D and Din)
        frame_ok = (D % 16 == 0 and self.Din % 8 == 0 and D <= 2048 and self.Din <= 2048
                    and dtype in (torch.float32, torch.bfloat16))
        if engine == "auto":
            engine = "frame" if frame_ok else "library"
        if engine == "frame" and not frame_ok:
            raise ValueError("engine='frame' needs hidden_dim % 16 == 0, input width % 8 == 0, "
                             "both <= 2048, and fp32 / bf16 weights")
        self.engine = engine
        if schedule not in ("wavefront", "frame"):
            raise ValueError("schedule must be 'wavefront' or 'frame'")
        # wavefront: the frame engine's block as stages over (frame, layer) (_block_wavefront)
        self.schedule = schedule if engine == "frame" else "frame"
        z = lambda *s, dt=dtype: torch.zeros(*s, dtype=dt, device=dev)   # noqa: E731
        if engine == "frame":
            f32 = torch.float32
            fb = lambda t: t.detach().float().contiguous()   # noqa: E731
            for e, cell in zip(self.layers, model.layers):
                e["b_in"] = fb(cell.input_proj.bias)
                e["b_g"] = fb(cell.W_fused.bias[D:]) if cfg.fused_ops else fb(torch.cat(
                    [m.bias for m in (cell.W_z, cell.W_k, cell.W_v, cell.W_decay)]))
                if not cfg.fused_ops:
                    e["b_h"] = fb(cell.W_h.bias)
            self.b_out = fb(model.output_proj.bias)
            self.x = z(K, B, self.Din, dt=f32)
            self.mask = torch.ones(K, B, dtype=f32, device=dev)
            self.fa, self.fz, self.fy, self.fhp = (z(B, D, dt=f32) for _ in range(4))
            self.st_a = z((D + 31) // 32, B, 4, dt=f32)   # (one record per 32 columns)
            self.st_z = z(D // 16, B, 4, dt=f32)
            self.st_h = z(D // 16, B, 4, dt=f32)
            self.xo = [z(B, D, dt=f32) for _ in range(self.L)]
            self.h = [z(B, D, dt=f32) for _ in range(self.L)]
            self.s = [z(B, D, dt=f32) for _ in range(self.L)]
            if self.schedule == "wavefront":
                # the layers of a stage run at once: each its own scratch; the last layer's
                # output per frame, for one output projection over the block
                self.wf = [dict(fa=z(B, D, dt=f32), fz=z(B, D, dt=f32), fy=z(B, D, dt=f32),
                                fhp=z(B, D, dt=f32), st_a=z((D + 31) // 32, B, 4, dt=f32),
                                st_z=z(D // 16, B, 4, dt=f32), st_h=z(D // 16, B, 4, dt=f32))
                           for _ in range(self.L)]
                self.xlast = z(K, B, D, dt=f32)
            self.logits = z(K, B, self.V, dt=f32)
            self.emit = torch.full((K, B), -1, dtype=torch.int32, device=dev)
            self.prev = torch.full((B,), -1, dtype=torch.int32, device=dev)
            self.graph = None
            if graph:
                self._capture()
            self.reset()
            return
        ng = 5 if cfg.fused_ops else 4
        self.x = z(K, B, self.Din)
        self.mask = torch.ones(K, B, dtype=torch.float32, device=dev)
        self.a, self.u, self.g = z(B, D), z(B, D), z(B, ng * D)
        self.y, self.hp = z(B, D), z(B, D)
        self.xo = [z(B, D) for _ in range(self.L)]
        self.h = [z(B, D, dt=torch.float32) for _ in range(self.L)]
        self.s = [z(B, D, dt=torch.float32) for _ in range(self.L)]
        self.logits = z(K, B, self.V)
        self.emit = torch.full((K, B), -1, dtype=torch.int32, device=dev)
        self.prev = torch.full((B,), -1, dtype=torch.int32, device=dev)
        self.graph = None
        if graph:
            self._capture()
        self.reset()

    # ------------------------------------------------------------------------------ frame --
    def _frame_fused_chain(self, j):
        """One frame on csrc/lucy_frame.hip's fused kernels (engine="frame")."""
        cfg, m, D = self.cfg, self.mask[j], self.D
        inp = self.x[j]
        for l, e in enumerate(self.layers):
            ln = e["ln_in"] is not None
            nst_a = (D + 31) // 32
            ops.lucy_frame_gemm(ops.FRAME_STATS if ln else ops.FRAME_PLAIN, inp, e["w_in"], e["b_in"],
                                self.fa, st_out=self.st_a[:nst_a] if ln else None)
            lnin = dict(ln=e["ln_in"], st_in=self.st_a[:nst_a]) if ln else {}
            if cfg.fused_ops:
                ops.lucy_frame_gemm(ops.FRAME_CELL_FUSED, self.fa, e["w_g"], e["b_g"], self.fhp,
                                    st_out=self.st_h, z=self.fz, st_z=self.st_z, s=self.s[l],
                                    mask=m, **lnin)
                st_h = self.st_h
            else:
                ops.lucy_frame_gemm(ops.FRAME_CELL_UNFUSED, self.fa, e["w_g"], e["b_g"], self.fy,
                                    z=self.fz, st_z=self.st_z, s=self.s[l], mask=m, **lnin)
                lnh = e["lnh"] is not None
                st_h = self.st_h[:nst_a]
                ops.lucy_frame_gemm(ops.FRAME_STATS if lnh else ops.FRAME_PLAIN, self.fy, e["w_h"],
                                    e["b_h"], self.fhp, st_out=st_h if lnh else None)
            ops.lucy_frame_cellb(self.fz, self.fhp, self.h[l], self.xo[l], st_z=self.st_z,
                                 st_h=st_h, lnz=e["lnz"], lnh=e["lnh"], mask=m)
            inp = self.xo[l]
        ops.lucy_frame_gemm(ops.FRAME_PLAIN, inp, self.w_out, self.b_out, self.logits[j])
        ops.ctc_greedy_step(self.logits[j], self.prev, self.emit[j], mask=m, blank=self.blank)

    def _frame(self, j):
        if self.engine == "frame":
            return self._frame_fused_chain(j)
        cfg, m = self.cfg, self.mask[j]
        inp = self.x[j]
        for l, e in enumerate(self.layers):
            torch.addmm(e["b_in"], inp, e["w_in"].t(), out=self.a)
            u = self.a
            if e["ln_in"] is not None:
                ops.lucy_step_ln(self.a, *e["ln_in"], self.u)
                u = self.u
            torch.addmm(e["b_g"], u, e["w_g"].t(), out=self.g)
            if cfg.fused_ops:
                ops.lucy_step_cell(ops.STEP_FUSED, self.g, self.h[l], self.s[l], self.xo[l],
                                   e["lnz"], e["lnh"], mask=m)
            else:
                ops.lucy_step_cell(ops.STEP_UNFUSED_A, self.g, self.h[l], self.s[l], self.y,
                                   e["lnz"], e["lnh"], u=u, mask=m)
                torch.addmm(e["b_h"], self.y, e["w_h"].t(), out=self.hp)
                ops.lucy_step_cell(ops.STEP_UNFUSED_B, self.g, self.h[l], self.s[l], self.xo[l],
                                   e["lnz"], e["lnh"], hp=self.hp, mask=m)
            inp = self.xo[l]
        torch.addmm(self.b_out, inp, self.w_out.t(), out=self.logits[j])
        ops.ctc_greedy_step(self.logits[j], self.prev, self.emit[j], mask=m, blank=self.blank)

    def _block_wavefront(self):
        """The frame engine's block as K + L - 1 stages: stage tau runs layer l of frame tau - l
        for every l at once (layer l of frame j needs layer l - 1 of frame j, from stage tau - 1,
        and layer l of frame j - 1, from stage tau - 1: its state).  A stage is the four kernels
        of a layer, each ONE launch over the stage's layers (sc_lucy_frame_gemm_multi /
        _cellb_multi); then one output projection over the K frames and one greedy launch.
        4 (K + L - 1) + 2 launches per block instead of K (4 L + 2), the same arithmetic per
        (frame, layer) as _frame_fused_chain.  Layer l's input xo[l - 1] is read by the stage's
        first launch and rewritten (next frame) by its last, so one buffer per layer suffices."""
        cfg, D, K, L = self.cfg, self.D, self.K, self.L
        stream = ops._lib.stream_of(self.x)
        wdt = self.w_out.dtype
        nst_a = (D + 31) // 32
        for tau in range(K + L - 1):
            act = [(l, tau - l) for l in range(L) if 0 <= tau - l < K]
            ln = self.layers[0]["ln_in"] is not None
            inproj, gates, whs, cells = [], [], [], []
            for l, j in act:
                e, sc, m = self.layers[l], self.wf[l], self.mask[j]
                inp = self.x[j] if l == 0 else self.xo[l - 1]
                inproj.append(ops.frame_gemm_job(inp, e["w_in"], e["b_in"], sc["fa"],
                                                 st_out=sc["st_a"][:nst_a] if ln else None))
                lnin = dict(ln=e["ln_in"], st_in=sc["st_a"][:nst_a]) if ln else {}
                if cfg.fused_ops:
                    gates.append(ops.frame_gemm_job(sc["fa"], e["w_g"], e["b_g"], sc["fhp"],
                                                    st_out=sc["st_h"], z=sc["fz"], st_z=sc["st_z"],
                                                    s=self.s[l], mask=m, **lnin))
                    st_h = sc["st_h"]
                else:
                    gates.append(ops.frame_gemm_job(sc["fa"], e["w_g"], e["b_g"], sc["fy"],
                                                    z=sc["fz"], st_z=sc["st_z"], s=self.s[l],
                                                    mask=m, **lnin))
                    lnh = e["lnh"] is not None
                    st_h = sc["st_h"][:nst_a]
                    whs.append(ops.frame_gemm_job(sc["fy"], e["w_h"], e["b_h"], sc["fhp"],
                                                  st_out=st_h if lnh else None))
                out = self.xlast[j] if l == L - 1 else self.xo[l]
                cells.append(ops.frame_cell_job(sc["fz"], sc["fhp"], self.h[l], out,
                                                st_z=sc["st_z"], st_h=st_h, lnz=e["lnz"],
                                                lnh=e["lnh"], mask=m))
            ops.lucy_frame_gemm_multi(ops.FRAME_STATS if ln else ops.FRAME_PLAIN, wdt, inproj, stream)
            ops.lucy_frame_gemm_multi(ops.FRAME_CELL_FUSED if cfg.fused_ops else ops.FRAME_CELL_UNFUSED,
                                      wdt, gates, stream)
            if whs:
                lnh = self.layers[0]["lnh"] is not None
                ops.lucy_frame_gemm_multi(ops.FRAME_STATS if lnh else ops.FRAME_PLAIN, wdt, whs,
                                          stream)
            ops.lucy_frame_cellb_multi(cells, stream)
        ops.lucy_frame_gemm(ops.FRAME_PLAIN, self.xlast.view(K * self.B, D), self.w_out, self.b_out,
                            self.logits.view(K * self.B, self.V))
        ops.ctc_greedy_frames(self.logits, self.prev, self.emit, mask=self.mask, blank=self.blank)

    def _block(self):
        if self.schedule == "wavefront":
            return self._block_wavefront()
        for j in range(self.K):
            self._frame(j)

    def _capture(self):
        side = torch.cuda.Stream(self.x.device)
        side.wait_stream(torch.cuda.current_stream(self.x.device))
        with torch.cuda.stream(side):   # warm-up: library workspaces, kernel loading
            self._block()
        torch.cuda.current_stream(self.x.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._block()

    # ------------------------------------------------------------------------------- API ---
    def reset(self, hidden_states=None, streams=None):
        """Start streams afresh: state from ``hidden_states`` ((h list, s list) of [B,D], as the
        reference's forward takes) or zero, prev token = none.  ``streams``: index tensor/list
        of the streams to reset (default all)."""
        idx = slice(None) if streams is None else torch.as_tensor(streams, device=self.x.device)
        for l in range(self.L):
            for buf, src in ((self.h[l], None if hidden_states is None else hidden_states[0][l]),
                             (self.s[l], None if hidden_states is None else hidden_states[1][l])):
                if src is None:
                    buf[idx] = 0.0
                else:
                    buf[idx] = src.to(buf.device, torch.float32)[idx]
        self.prev[idx] = -1

    def state(self):
        """(h list, s list) fp32 copies — the reference's (h, s) return (lucyrnn.py:188-189)."""
        return [t.clone() for t in self.h], [t.clone() for t in self.s]

    def step(self, x, mask=None):
        """Advance every stream by K = frames_per_call model frames.  x [B, K, input_dim *
        stack_order] (already stacked); mask [B, K] (bool/float, None = all live).  Returns
        emit int32 [B, K] on the device: the token decoder.py appends at that frame, or -1.
        The logits of the block stay in ``self.logits`` ([K, B, V])."""
        self.x.copy_(x.transpose(0, 1))
        if mask is None:
            self.mask.fill_(1.0)
        else:
            self.mask.copy_(mask.transpose(0, 1))
        if self.graph is not None:
            self.graph.replay()
        else:
            self._block()
        return self.emit.t()

    def decode(self, feats, masks=None, return_logits=False):
        """Whole utterances through the streaming path: feats [B, T, input_dim] raw frames,
        stacked as the model does (lucyrnn.py:92-99: the tail T % stack_order is dropped, a
        stacked frame is live when all its frames are).  Returns the decoder.py token lists
        (and logits [B, T', V] if asked).  One host sync at the end."""
        B, T, F = feats.shape
        k = self.cfg.stack_order
        Tt = T - T % k
        x = feats[:, :Tt].reshape(B, Tt // k, F * k)
        m = None
        if masks is not None:
            m = masks.reshape(B, -1)[:, :Tt].reshape(B, Tt // k, k).all(-1).float()
        T2 = x.shape[1]
        emits, logits = [], []
        for t0 in range(0, T2, self.K):
            n = min(self.K, T2 - t0)
            xb = torch.zeros(B, self.K, x.shape[2], dtype=self.dtype, device=self.x.device)
            xb[:, :n] = x[:, t0:t0 + n]
            mb = torch.zeros(B, self.K, device=self.x.device)   # padding frames are masked out
            mb[:, :n] = 1.0 if m is None else m[:, t0:t0 + n]
            emits.append(self.step(xb, mb)[:, :n].clone())
            if return_logits:
                logits.append(self.logits[:n].transpose(0, 1).clone())
        em = torch.cat(emits, 1).cpu() if emits else torch.zeros(B, 0, dtype=torch.int32)
        toks = [[int(t) for t in row if t >= 0] for row in em]
        if return_logits:
            return toks, torch.cat(logits, 1) if logits else None
        return toks
