"""Device-resident greedy decoding for one batch (WhisperDecoder + GenerationMixin._sample).

A ``DecodeSession`` owns the static caches and step buffers of one batch:
  * cross K/V of every layer ([2L][B][H][1500][64], one GEMM, TF modeling_whisper.py:323-335), per item
    (beams share it);
  * self K/V static cache [L][B][H][448][64] (replaces DynamicLayer's torch.cat growth,
    TF/cache_utils.py:127-145);
  * ids [B][448] int64, cur_len, unfinished flags -- all on device, advanced by kw_greedy_step.
The prefill (prompt of P tokens) runs eagerly; the single-token step (embedding + 32 x 8 kernels +
LM head with the final LayerNorm fused + sampler) is captured once into a hipGraph (torch.cuda.CUDAGraph) and replayed: the step
reads its position from device memory, so one graph serves every step.  The host only polls the
device unfinished-row count a few steps behind the GPU (no per-step sync).  Graphs are captured with
capture_error_mode="thread_local", so another host thread (another batch in flight on its own stream,
WhisperEngine.lane()) may keep launching while one session captures.  Captures themselves are serialised by one
process-wide lock (``CAPTURE_LOCK``): ``torch.cuda.graph.__enter__`` synchronises the whole device and empties the
allocator cache, which must not run inside another thread's capture; session creation (allocations) takes the same
lock.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from . import _lib as L
from . import ops

_HD = 64
T_MAX = 448
# serialises every hipGraph capture and every session allocation of the process (lanes capture on host threads)
CAPTURE_LOCK = threading.RLock()


_CAPTURE_STREAMS = {}  # device -> the stream every capture of the process runs on (captures are serialised)


def capture_graph(fn, dev) -> torch.cuda.CUDAGraph:
    """Capture ``fn``'s launches into a new graph on a side stream of its own (L.new_stream: never a pooled stream
    another thread may be launching on), under CAPTURE_LOCK."""
    with CAPTURE_LOCK:
        g = torch.cuda.CUDAGraph()
        key = torch.device(dev).index if torch.device(dev).index is not None else torch.cuda.current_device()
        side = _CAPTURE_STREAMS.get(key)
        if side is None:
            side = _CAPTURE_STREAMS[key] = L.new_stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
            fn()
        torch.cuda.current_stream(dev).wait_stream(side)
    return g


class DecodeSession:
    def __init__(self, eng, B: int, enc: torch.Tensor | None = None, beams: int = 1):
        """B batch items decoded as R = B * beams running rows (item-major); cross K/V per item."""
        s = eng.shape
        self.eng, self.B, self.nb = eng, B, beams
        R = self.R = B * beams
        dev, dt = eng.device, eng.dtype
        d, H, Ld = s.d_model, eng.H, s.decoder_layers
        self.T = s.max_source_positions
        self.cross = torch.empty((2 * Ld, B, H, self.T, _HD), device=dev, dtype=dt)
        self.kc = torch.zeros((Ld, R, H, T_MAX, _HD), device=dev, dtype=dt)
        self.vc = torch.zeros((Ld, R, H, T_MAX, _HD), device=dev, dtype=dt)
        self.ids = torch.zeros((R, T_MAX + 1), device=dev, dtype=torch.int64)
        # beam search: cache row holding position p of row r's history (beams share a prefix)
        self.bp = torch.zeros((R, T_MAX), device=dev, dtype=torch.int32) if beams > 1 else None
        self.cur_len = torch.zeros((1,), device=dev, dtype=torch.int32)
        self.unfinished = torch.ones((R,), device=dev, dtype=torch.int32)
        self.counter = torch.zeros((1,), device=dev, dtype=torch.int32)
        self.n_unfinished = torch.zeros((1,), device=dev, dtype=torch.int32)
        self.logits = torch.empty((R, s.vocab_size), device=dev, dtype=torch.float32)
        self._bufs = {}
        self._plans = {}
        # split-K seam scratch shared by every decode linear of a step (stream-ordered; zeroed once)
        ws = 0
        if eng.packed:
            for n_, k_ in ((3 * d, d), (d, d), (s.decoder_ffn_dim, d), (d, s.decoder_ffn_dim), (s.vocab_size, d),
                           (H * d, _HD)):
                ws = max(ws, ops.dec_linear_workspace_bytes(n_, k_))
        self.lin_ws = torch.zeros(((ws + 3) // 4,), device=dev, dtype=torch.float32) if ws else None
        self.self_ws = torch.zeros((ops.self_attn_workspace_bytes(R, H, T_MAX) + 3) // 4, device=dev,
                                   dtype=torch.float32)
        # fused self-attention block (kw_dec_qkv_self): greedy rows of the bf16 engine, <= 32 per session, steps
        # at positions < 256 (decided per generate call); its granule workspace is zeroed once, every launch
        # re-arms it
        self.qs_ok = (eng.packed and beams == 1 and eng.fuse_qkv_self and R <= 32
                      and ops.qkv_self_supported(R, d, H))
        self.qs_ws = torch.zeros(((ops.qkv_self_workspace_bytes(R, d) + 3) // 4,), device=dev,
                                 dtype=torch.float32) if self.qs_ok else None
        self.fused_last = False  # whether the last step plan built / replayed used kw_dec_qkv_self
        # fused cross-attention query + step (kw_dec_xq_cross): one query row per item (greedy), any position
        self.xc_ok = (eng.packed and beams == 1 and eng.fuse_xq_cross and R <= 32
                      and ops.xq_cross_supported(R, d, H, self.T))
        self.xc_ws = torch.zeros(((ops.xq_cross_workspace_bytes(R, d, H, self.T) + 3) // 4,), device=dev,
                                 dtype=torch.float32) if self.xc_ok else None
        self._graph = None
        self._graph_key = None
        self._cross_key = None
        # split-row sampler partials + per-row arrival counters (zeroed once; kernels leave them zeroed)
        self.samp_ws = torch.zeros((ops.greedy_step_workspace_bytes(R) + 3) // 4, device=dev, dtype=torch.float32)
        self._greedy_cfg = {}
        self._pinned = None
        self._lmg_ws = None  # kw_dec_lm_greedy's partials + arrival counter (zeroed once; launches re-arm it)
        self.lm_greedy_last = False
        self.last_steps = 0
        if enc is not None:
            self.set_encoder_output(enc)

    # ------------------------------------------------------------------------------------------
    def set_encoder_output(self, enc: torch.Tensor, key=None) -> None:
        """Project ``enc`` into every layer's cross K/V.  ``key`` (optional) names the encoder output: a
        repeat call with the key of the K/V already held skips the projection (the v3 multi-task loop
        decodes several prompts against one encoder pass, run_pseudo_labelling_v3.py:309-321)."""
        if key is not None and key == self._cross_key:
            return
        self.eng.cross_kv(enc, self.B, out=self.cross)
        self._cross_key = key

    def _row_view(self, r0: int, r1: int) -> "DecodeSession":
        """A session over greedy rows [r0, r1) of this one: its ids / caches / cross K/V / logits are row slices
        of this session's, its activation buffers and launch workspaces its own (so two views can run at once).
        Every decode op's per-row arithmetic is independent of the other rows, so a view computes bitwise what
        the full session computes for those rows."""
        v = object.__new__(DecodeSession)
        v.eng, v.nb, v.B, v.R, v.T = self.eng, 1, r1 - r0, r1 - r0, self.T
        v.cross, v.kc, v.vc = self.cross[:, r0:r1], self.kc[:, r0:r1], self.vc[:, r0:r1]
        v.ids, v.bp, v.cur_len, v.logits = self.ids[r0:r1], None, self.cur_len, self.logits[r0:r1]
        v._bufs, v._plans = {}, {}
        v.lin_ws = torch.zeros_like(self.lin_ws) if self.lin_ws is not None else None
        v.self_ws = torch.zeros_like(self.self_ws)
        v.qs_ok = v.xc_ok = False
        v.qs_ws = v.xc_ws = None
        return v

    def _prefill_parts(self, parts: int):
        """Row views for a prefill split over ``parts`` side streams (greedy rows only), cached."""
        key = ("views", parts)
        if key not in self._plans:
            R = self.R
            sizes = [R // parts + (1 if i < R % parts else 0) for i in range(parts)]
            views, r0 = [], 0
            for n in sizes:
                views.append(self._row_view(r0, r0 + n))
                r0 += n
            # (streams of their own: a captured prefill forks into them, L.new_stream)
            self._plans[key] = (views, [L.new_stream(self.eng.device, owner=self) for _ in range(parts)])
        return self._plans[key]

    def _run_prefill(self, P: int, parts: int) -> None:
        """The prompt's forward pass (prefill) as ``parts`` row blocks on side streams, their launches issued in
        lockstep: each block's kernels are latency-bound chains on few CUs, and two of them overlap (the
        encoder's split, engine._encode_split).  Joined on the current stream before the sampler."""
        if parts <= 1 or self.nb != 1 or self.R < 2 * parts:
            self._run(self._step_plans(P))
            return
        views, streams = self._prefill_parts(parts)
        seqs = [v._step_plans(P) for v in views]
        cur = torch.cuda.current_stream(self.eng.device)
        for st in streams:
            st.wait_stream(cur)
        for j in range(len(seqs[0])):
            for v, seq, st in zip(views, seqs, streams):
                with torch.cuda.stream(st):
                    v._run([seq[j]])
        for st in streams:
            cur.wait_stream(st)

    def _buffers(self, q: int):
        if q not in self._bufs:
            s, dev, dt = self.eng.shape, self.eng.device, self.eng.dtype
            d, rows = s.d_model, self.R * q
            self._bufs[q] = dict(
                h=torch.empty((rows, d), device=dev, dtype=torch.float32),
                x=torch.empty((rows, d), device=dev, dtype=dt),
                qkv=torch.empty((rows, 3 * d), device=dev, dtype=dt),
                attn=torch.empty((rows, d), device=dev, dtype=dt),
                qx=torch.empty((rows, d), device=dev, dtype=dt),
                ffn=torch.empty((rows, s.decoder_ffn_dim), device=dev, dtype=dt),
                # cross-attention partials + arrival counters (must start zeroed; kernels leave them zeroed)
                ws=torch.zeros((ops.cross_attn_workspace_bytes(self.B, q * self.nb, self.eng.H, _HD, self.T) // 4 + 1,),
                               device=dev, dtype=torch.float32),
            )
            if self.eng.packed:  # bf16 mirror of the residual stream (the LayerNorm-fused linears' operand)
                self._bufs[q]["hb"] = torch.empty((rows, d), device=dev, dtype=torch.bfloat16)
        return self._bufs[q]

    def _gemm(self, A, W, C, M, N, K, **kw):
        """f32 parity-mode linear (kw_gemm)."""
        return [ops.GemmPlan(A, W, C, M, N, K, **kw)]

    def _step_plans(self, q: int, fused: bool = False):
        """The decoder forward for q new positions per row (q = prompt length for the prefill, 1 after).
        ``fused`` (q == 1): each layer's LayerNorm-fused QKV projection and self-attention step as ONE
        kw_dec_qkv_self launch (caches bitwise the two-launch plan's, attention within bf16 rounding) -- for steps at positions < 256 only."""
        fused = bool(fused and q == 1 and self.qs_ok)
        key = (q, fused)
        if key in self._plans:
            return self._plans[key]
        eng, s = self.eng, self.eng.shape
        b = self._buffers(q)
        d, H, B = s.d_model, eng.H, self.R  # B: running rows
        rows = B * q
        scale = _HD ** -0.5
        eps = s.layer_norm_eps
        if eng.packed:
            # bf16 path: every decoder LayerNorm is fused into the linear that consumes it
            # (operand = the bf16 residual mirror hb, its rows' statistics computed in that kernel); the
            # residual-add linears update h and hb.
            hb, h = b["hb"], b["h"]
            ws = self.lin_ws
            lin = ops.DecLinearPlan
            seq = [("embed", q, h, hb)]
            for li, lay in enumerate(eng.dec_layers):
                if fused:
                    seq.append(ops.QkvSelfPlan(hb, lay["qkv_w"], rows, d, H, ln=(eps, lay["qkv_cs"]), bias=lay["qkv_b"],
                                               scale=scale, k_cache=self.kc[li], v_cache=self.vc[li], t_max=T_MAX,
                                               cur_len=self.cur_len, out=b["attn"], workspace=self.qs_ws))
                else:
                    seq.append(lin(hb, lay["qkv_w"], rows, 3 * d, d, ln=(eps, lay["qkv_cs"]), bias=lay["qkv_b"],
                                   C=b["qkv"], scale=scale, scale_cols=d, workspace=ws, tag="qkv"))
                    seq.append(("self", q, b["qkv"], li, b["attn"]))
                seq.append(lin(b["attn"], lay["o_w"], rows, d, d, bias=lay["o_b"], resid=(h, hb, d, 0), workspace=ws,
                               tag="o"))
                if q == 1 and self.xc_ok:
                    seq.append(ops.XqCrossPlan(hb, lay["xq_w"], rows, d, H, ln=(eps, lay["xq_cs"]), bias=lay["xq_b"],
                                               scale=scale, k=self.cross[2 * li], v=self.cross[2 * li + 1], S=self.T,
                                               out=b["attn"], workspace=self.xc_ws))
                else:
                    seq.append(lin(hb, lay["xq_w"], rows, d, d, ln=(eps, lay["xq_cs"]), bias=lay["xq_b"],
                                   C=b["qx"], scale=scale, scale_cols=d, workspace=ws, tag="xq"))
                    seq.append(("cross", q, b["qx"], li, b["attn"], b["ws"]))
                seq.append(lin(b["attn"], lay["xo_w"], rows, d, d, bias=lay["xo_b"], resid=(h, hb, d, 0),
                               workspace=ws, tag="xo"))
                seq.append(lin(hb, lay["fc1_w"], rows, s.decoder_ffn_dim, d, ln=(eps, lay["fc1_cs"]),
                               bias=lay["fc1_b"], C=b["ffn"], gelu=True, workspace=ws, tag="fc1"))
                seq.append(lin(b["ffn"], lay["fc2_w"], rows, d, s.decoder_ffn_dim, bias=lay["fc2_b"],
                               resid=(h, hb, d, 0), workspace=ws, tag="fc2"))
            # final LayerNorm (folded into the packed LM head) + proj_out on the last position of every row
            seq.append(lin(hb, eng.lm_w, B, s.vocab_size, d, ldx=q * d, x_offset=(q - 1) * d,
                           ln=(eps, eng.lm_cs), bias=eng.lm_b, C=self.logits, workspace=ws, tag="lm_head"))
            self._plans[key] = seq
            return seq
        seq = [("embed", q, b["h"])]
        for li, lay in enumerate(eng.dec_layers):
            seq.append(("ln", b["h"], lay["ln1_g"], lay["ln1_b"], b["x"]))
            seq += self._gemm(b["x"], lay["qkv_w"], b["qkv"], rows, 3 * d, d, bias=lay["qkv_b"], scale=scale,
                              scale_cols=d)
            seq.append(("self", q, b["qkv"], li, b["attn"]))
            seq += self._gemm(b["attn"], lay["o_w"], b["h"], rows, d, d, bias=lay["o_b"], epilogue=L.KW_EPI_RESID)
            seq.append(("ln", b["h"], lay["ln2_g"], lay["ln2_b"], b["x"]))
            seq += self._gemm(b["x"], lay["xq_w"], b["qx"], rows, d, d, bias=lay["xq_b"], scale=scale, scale_cols=d)
            seq.append(("cross", q, b["qx"], li, b["attn"], b["ws"]))
            seq += self._gemm(b["attn"], lay["xo_w"], b["h"], rows, d, d, bias=lay["xo_b"], epilogue=L.KW_EPI_RESID)
            seq.append(("ln", b["h"], lay["ln3_g"], lay["ln3_b"], b["x"]))
            seq += self._gemm(b["x"], lay["fc1_w"], b["ffn"], rows, s.decoder_ffn_dim, d, bias=lay["fc1_b"],
                              gelu=True)
            seq += self._gemm(b["ffn"], lay["fc2_w"], b["h"], rows, d, s.decoder_ffn_dim, bias=lay["fc2_b"],
                              epilogue=L.KW_EPI_RESID)
        seq.append(("ln", b["h"], eng.dec_ln_g, eng.dec_ln_b, b["x"]))
        # LM head on the last position of every row (proj_out tied to embed_tokens, f32 logits)
        seq += self._gemm(b["x"], eng.lm_w, self.logits, B, s.vocab_size, d, lda=q * d, a_offset=(q - 1) * d)
        self._plans[key] = seq
        return seq

    def _run(self, seq):
        eng, s = self.eng, self.eng.shape
        H, B = eng.H, self.R
        for p in seq:
            if not isinstance(p, tuple):
                p()
                continue
            k = p[0]
            if k == "ln":
                ops.layernorm(p[1], p[2], p[3], s.layer_norm_eps, p[4])
            elif k == "embed":
                ops.embed(self.ids, B, p[1], self.cur_len, eng.tok_emb, eng.dec_pos, p[2], p[3] if len(p) > 3 else None)
            elif k == "self":
                _, q, qkv, li, out = p
                ops.self_attn_step(qkv, B, q, H, _HD, self.kc[li], self.vc[li], T_MAX, self.cur_len, out, self.self_ws,
                                   bp=self.bp if q == 1 else None)
            elif k == "cross":  # rows b*nb*q + (beam*q + i) attend to item b's K/V
                _, q, qx, li, out, ws = p
                ops.cross_attn_step(qx, self.B, q * self.nb, H, _HD, self.cross[2 * li], self.cross[2 * li + 1],
                                    self.T, out, ws)

    # ------------------------------------------------------------------------------------------
    def status_words(self):
        """(entry point, workspace, byte offset) of every in-launch hand-off status word this session's launches
        can set (include/kwhisper.h kw_*_status_offset): the fused self block, the fused cross block and the
        unfused cross-attention's combine, one per activation-buffer size."""
        s, H = self.eng.shape, self.eng.H
        out = []
        if self.qs_ws is not None:
            out.append(("kw_dec_qkv_self", self.qs_ws, ops.status_offset("qkv_self", self.R, s.d_model)))
        if self.xc_ws is not None:
            out.append(("kw_dec_xq_cross", self.xc_ws, ops.status_offset("xq_cross", self.R, s.d_model, H, self.T)))
        for q, b in self._bufs.items():
            out.append(("kw_cross_attn_step", b["ws"], ops.status_offset("cross_attn", self.B, q * self.nb, H, _HD,
                                                                         self.T)))
        return out

    def check_handoffs(self) -> None:
        """After the stream is synchronized: raise ``KWError`` if any launch of this session had an in-launch
        hand-off time out (its rows were written as NaN, so its tokens are wrong).  One small device-to-host copy;
        on failure every such workspace is zero-filled (re-armed) first, so the session stays usable."""
        words = self.status_words()
        if not words:
            return
        st = torch.stack([ws.view(torch.int32)[off // 4] for _, ws, off in words]).cpu().tolist()
        bad = [name for (name, _, _), v in zip(words, st) if v != 0]
        if bad:
            for _, ws, _ in words:
                ws.zero_()
            raise L.KWError(f"{', '.join(sorted(set(bad)))}: an in-launch hand-off timed out (a kernel protocol "
                            "failure); the rows it fed are NaN, so this call's tokens are invalid")

    def forward_logits(self, prompt: torch.Tensor) -> torch.Tensor:
        """Prefill only: logits (B, V) for the last prompt position (detect_language)."""
        P = prompt.shape[1]
        self.ids[:, :P].copy_(prompt)
        self.cur_len.fill_(P)
        self._run(self._step_plans(P))
        return self.logits

    def teacher_forced_logits(self, seq: torch.Tensor, P: int) -> torch.Tensor:
        """Raw logits (B, T-P+1, V) predicting seq[:, P:] and one more, feeding the reference tokens
        (validation utility: compares the decoder step with a reference's per-step logits)."""
        B, T = seq.shape
        seq = seq.to(self.eng.device)
        self.ids.zero_()
        self.ids[:, :T].copy_(seq)
        self.cur_len.fill_(P)
        out = []
        self._run(self._step_plans(P))
        out.append(self.logits.clone())
        step = self._step_plans(1, fused=T <= 256)
        for t in range(P, T):
            self.cur_len.fill_(t + 1)
            self._run(step)
            out.append(self.logits.clone())
        return torch.stack(out, 1)

    def _pinned_slots(self, n: int) -> torch.Tensor:
        if self._pinned is None or self._pinned.numel() < n:
            self._pinned = torch.zeros((n,), dtype=torch.int32).pin_memory()
        return self._pinned

    @staticmethod
    def _poll(pinned, events, rep, lag, flag) -> bool:
        """Queue a copy of the device ``flag`` (unfinished rows / beam "go") into pinned slot ``rep % (lag + 1)``
        behind the replay just issued, then read the copy issued ``lag`` replays ago; True once that count is 0
        (every later replay is then a no-op on device: finished rows only append pad).  The slot first gets a -1
        sentinel, so only a count a copy actually delivered can stop the loop (r03al)."""
        slot = rep % (lag + 1)
        pinned[slot] = -1
        pinned[slot: slot + 1].copy_(flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        events.append((ev, slot))
        if len(events) > lag:
            e0, s0 = events.pop(0)
            e0.synchronize()
            return int(pinned[s0]) == 0
        return False

    def generate(self, prompt: torch.Tensor, gen, *, max_length: int, return_timestamps: bool,
                 check_every: int = 4, use_graph: bool = True, record_scores: bool = False):
        """Greedy loop of GenerationMixin._sample (TF/generation/utils.py:2783-2941).

        Returns host int64 ids (B, L) including the prompt, with L exactly the length the reference
        loop stops at (all rows finished or max_length)."""
        B = self.B
        P = prompt.shape[1]
        if P + 1 > T_MAX + 1 or max_length > T_MAX:
            raise ValueError(f"max_length {max_length} exceeds max_target_positions {T_MAX}")
        dev = self.eng.device
        self.ids.zero_()
        self.ids[:, :P].copy_(prompt.to(dev))
        self.cur_len.fill_(P)
        self.unfinished.fill_(1)
        self.counter.zero_()
        self.n_unfinished.fill_(B)
        # the sampler plan, its processor tables and the captured step graph are kept per configuration:
        # a repeat call (the next batch) replays the same graph (no re-capture)
        key = (max_length, P, bool(return_timestamps), tuple(gen.suppress_tokens or ()),
               tuple(gen.begin_suppress_tokens or ()), gen.timestamp_begin, gen.no_timestamps_token_id,
               gen.eos_token_id, gen.pad_token_id, gen.max_initial_timestamp_index, bool(record_scores),
               self.eng.prefill_streams, self.eng.fuse_lm_greedy)
        cfg = self._greedy_cfg.get(key)
        if cfg is None:
            sup = torch.zeros((self.eng.shape.vocab_size,), dtype=torch.uint8)
            if gen.suppress_tokens:
                sup[torch.tensor(gen.suppress_tokens)] = 1
            sup = sup.to(dev)
            bsup = torch.tensor(gen.begin_suppress_tokens or [0], dtype=torch.int32, device=dev)
            nb = len(gen.begin_suppress_tokens or [])
            score_buf = torch.empty_like(self.logits) if record_scores else None
            sampler = ops.SamplerPlan(self.logits, sup, bsup if nb else None, self.ids, self.cur_len,
                                      self.unfinished, self.counter, self.n_unfinished,
                                      return_timestamps=return_timestamps, ts_begin=gen.timestamp_begin,
                                      no_ts_id=gen.no_timestamps_token_id, eos_id=gen.eos_token_id,
                                      pad_id=gen.pad_token_id, max_initial_ts=gen.max_initial_timestamp_index,
                                      max_length=max_length, begin_index=P, scores_out=score_buf,
                                      workspace=self.samp_ws)
            cfg = dict(sampler=sampler, score_buf=score_buf, graph=None)
            if len(self._greedy_cfg) >= 8:  # bound the cache (each entry may hold a graph)
                self._greedy_cfg.pop(next(iter(self._greedy_cfg)))
            self._greedy_cfg[key] = cfg
        sampler, score_buf = cfg["sampler"], cfg["score_buf"]
        self.scores = [] if record_scores else None
        # prefill (replayed from a graph cached with the configuration: ~260 launches otherwise go
        # through Python one by one)
        def prefill():
            self._run_prefill(P, self.eng.prefill_streams)
            sampler()

        pg = cfg.get("prefill_graph")
        if pg is None and use_graph and not record_scores:
            pg = cfg["prefill_graph"] = capture_graph(prefill, dev)
            # capture only records: the kernels have not run yet, and the state the prefill consumes
            # (ids, cur_len, counters) is untouched -- replay below
        if pg is not None and use_graph and not record_scores:
            pg.replay()
        else:
            prefill()
        if record_scores:
            self.scores.append((self.logits.clone(), score_buf.clone()))
        n_steps = max_length - P  # tokens the reference can add at most
        done = 1
        fused = max_length <= 256  # every step's position < 256 (kw_dec_qkv_self's key range)
        step_seq = self._step_plans(1, fused=fused)
        self.fused_last = bool(fused and self.qs_ok)
        # the step's LM head + greedy step as one launch (kw_dec_lm_greedy; no timestamps, no recorded scores)
        tail = sampler
        s = self.eng.shape
        if (self.eng.packed and self.nb == 1 and self.eng.fuse_lm_greedy and not return_timestamps and not record_scores
                and ops.lm_greedy_supported(B, s.vocab_size, s.d_model)):
            tail = cfg.get("lm_greedy")
            if tail is None:
                if self._lmg_ws is None:
                    self._lmg_ws = torch.zeros((ops.lm_greedy_workspace_bytes(B, s.vocab_size) + 3) // 4, device=dev,
                                               dtype=torch.float32)
                sa = sampler.args
                tail = cfg["lm_greedy"] = ops.LmGreedyPlan(
                    self._buffers(1)["hb"], self.eng.lm_w, B, s.vocab_size, s.d_model, ln=(s.layer_norm_eps, self.eng.lm_cs),
                    bias=self.eng.lm_b, suppress_mask=sampler._keep[1], begin_suppress=sampler._keep[2], ids=self.ids,
                    cur_len=self.cur_len, unfinished=self.unfinished, n_unfinished=self.n_unfinished, eos_id=sa.eos_id,
                    pad_id=sa.pad_id, max_length=sa.max_length, begin_index=sa.begin_index, workspace=self._lmg_ws)
            assert getattr(step_seq[-1], "tag", None) == "lm_head"
            step_seq = step_seq[:-1]
        self.lm_greedy_last = tail is not sampler

        def one_step():
            self._run(step_seq)
            tail()

        def capture(n):
            def steps():
                for _ in range(n):
                    one_step()
            return capture_graph(steps, dev)

        graph = cfg["graph"]
        if graph is None and use_graph and not record_scores and n_steps > 1:
            graph = cfg["graph"] = capture(1)
        # K (engine.steps_per_replay) steps per replay where K steps remain: one replay launch, unfinished-count
        # copy and event per K steps; every step reads its position from the device, so K steps in one graph are
        # the same K replays of the one-step graph
        K = max(1, int(self.eng.steps_per_replay))
        graph_k = cfg.get(("graph", K)) if K > 1 else None
        if K > 1 and graph_k is None and graph is not None and n_steps > K:
            graph_k = cfg[("graph", K)] = capture(K)
        if not use_graph:
            graph = graph_k = None
        self._graph, self._graph_key = graph, key
        lag = max(1, check_every // K) if graph_k is not None else check_every  # the same lag in steps
        pinned = self._pinned_slots(lag + 1)
        events = []
        rep = 0  # replays issued: slot rep % (lag + 1) is distinct over the lag + 1 copies in flight
        while done < n_steps:
            if graph_k is not None and done + K <= n_steps:
                graph_k.replay()
                done += K
            else:
                if graph is not None:
                    graph.replay()
                else:
                    one_step()
                done += 1
            if record_scores:
                self.scores.append((self.logits.clone(), score_buf.clone()))
            if self._poll(pinned, events, rep, lag, self.n_unfinished):
                break
            rep += 1
        self.last_steps = done  # steps issued (tests: the stop check fires within lag steps of the last EOS)
        torch.cuda.current_stream(dev).synchronize()  # (this stream only: other lanes keep running)
        self.check_handoffs()
        L_now = int(self.cur_len.item())
        ids = self.ids[:, :L_now].cpu().numpy()
        return _reference_length(ids, P, gen.eos_token_id, max_length)


    def generate_beam(self, prompt: torch.Tensor, gen, *, num_beams: int, max_length: int, return_timestamps: bool,
                      length_penalty: float = 1.0, early_stopping=False, check_every: int = 4, use_graph: bool = True):
        """``GenerationMixin._beam_search`` (TF/generation/utils.py:3208-3527) on device, num_return_sequences 1.

        ``prompt`` (B, P) per item.  Returns host int64 (B, P + generated) -- the best finished beam of each
        item, pad-filled, cropped to the batch's longest -- as the reference returns ``sequences``."""
        B, nb, R = self.B, self.nb, self.R
        if nb != num_beams or nb < 2:
            raise ValueError("session beam width mismatch")
        P = prompt.shape[1]
        if max_length > T_MAX:
            raise ValueError(f"max_length {max_length} exceeds max_target_positions {T_MAX}")
        dev = self.eng.device
        V = self.eng.shape.vocab_size
        fill = gen.pad_token_id if gen.pad_token_id is not None else gen.eos_token_id
        self.ids.zero_()
        self.ids[:, :P].copy_(prompt.to(dev).repeat_interleave(nb, 0))
        self.cur_len.fill_(P)
        self.bp.copy_(torch.arange(R, device=dev, dtype=torch.int32)[:, None].expand(R, T_MAX))
        # beam state, step plan and captured graphs are kept per configuration and re-initialised in
        # place, so a repeat call replays the same graphs (no re-capture, see generate)
        key = ("beam", max_length, P, bool(return_timestamps), float(length_penalty), str(early_stopping), fill,
               tuple(gen.suppress_tokens or ()), tuple(gen.begin_suppress_tokens or ()), gen.timestamp_begin,
               gen.no_timestamps_token_id, gen.eos_token_id, gen.max_initial_timestamp_index)
        cfg = self._greedy_cfg.get(key)
        if cfg is None:
            st = dict(
                ids=self.ids, bp=self.bp, cur_len=self.cur_len,
                run_scores=torch.empty((B * nb,), device=dev, dtype=torch.float32),
                fin_seq=torch.empty((B, nb, max_length), device=dev, dtype=torch.int64),
                fin_score=torch.empty((B, nb), device=dev, dtype=torch.float32),
                fin_len=torch.empty((B, nb), device=dev, dtype=torch.int32),
                fin_flag=torch.empty((B, nb), device=dev, dtype=torch.int32),
                unsat=torch.empty((B,), device=dev, dtype=torch.int32),
                counter=torch.zeros((1,), device=dev, dtype=torch.int32),
                go=torch.empty((1,), device=dev, dtype=torch.int32),
                done=torch.empty((1,), device=dev, dtype=torch.int32),
                item_flags=torch.empty((B, 3), device=dev, dtype=torch.int32),
                cand_val=torch.empty((R, 2 * nb), device=dev, dtype=torch.float32),
                cand_idx=torch.empty((R, 2 * nb), device=dev, dtype=torch.int32),
                lp_ws=torch.zeros(((ops.beam_logprobs_workspace_bytes(R) + 3) // 4,), device=dev, dtype=torch.float32),
            )
            sup = torch.zeros((V,), dtype=torch.uint8)
            if gen.suppress_tokens:
                sup[torch.tensor(gen.suppress_tokens)] = 1
            sup = sup.to(dev)
            bsup = torch.tensor(gen.begin_suppress_tokens or [0], dtype=torch.int32, device=dev)
            step = ops.BeamStepPlan(st, self.logits, sup, bsup if gen.begin_suppress_tokens else None,
                                    return_timestamps=return_timestamps, ts_begin=gen.timestamp_begin,
                                    no_ts_id=gen.no_timestamps_token_id, eos_id=gen.eos_token_id,
                                    max_initial_ts=gen.max_initial_timestamp_index, begin_index=P,
                                    max_length=max_length, fill_id=fill, length_penalty=length_penalty,
                                    early_stopping=early_stopping)
            cfg = dict(st=st, step=step, graph=None, prefill_graph=None)
            if len(self._greedy_cfg) >= 8:
                self._greedy_cfg.pop(next(iter(self._greedy_cfg)))
            self._greedy_cfg[key] = cfg
        st, step = cfg["st"], cfg["step"]
        st["run_scores"].view(B, nb).fill_(-1.0e9)
        st["run_scores"].view(B, nb)[:, 0] = 0.0
        st["fin_seq"].fill_(fill)
        st["fin_score"].fill_(-1.0e9)
        st["fin_len"].zero_()
        st["fin_flag"].zero_()
        st["unsat"].fill_(1)
        st["counter"].zero_()
        st["go"].fill_(1)
        st["done"].zero_()
        st["item_flags"].zero_()
        self._beam_state = st

        def prefill():
            self._run(self._step_plans(P))  # prefill on every running row (the reference expands x num_beams)
            step()

        step_seq = self._step_plans(1)

        def one_step():
            self._run(step_seq)
            step()

        def captured(name, fn):
            g = cfg[name]
            if g is None:
                g = cfg[name] = capture_graph(fn, dev)
            return g

        if use_graph:
            captured("prefill_graph", prefill).replay()
        else:
            prefill()
        graph = captured("graph", one_step) if use_graph else None
        pinned = self._pinned_slots(check_every + 1)
        events = []
        n = 1
        while n < max_length - P + 1:
            if graph is not None:
                graph.replay()
            else:
                one_step()
            if self._poll(pinned, events, n - 1, check_every, st["go"]):
                break
            n += 1
        torch.cuda.current_stream(dev).synchronize()  # (this stream only: other lanes keep running)
        self.check_handoffs()
        fin_len = st["fin_len"][:, 0].cpu().numpy()
        out = st["fin_seq"][:, 0].cpu().numpy()
        return out[:, : P + int(fin_len.max())]


def _reference_length(ids: np.ndarray, P: int, eos: int, max_length: int) -> np.ndarray:
    """Trim to the length at which the reference's while-loop would have stopped."""
    B, L_now = ids.shape
    stop = []
    for b in range(B):
        hit = np.nonzero(ids[b, P:] == eos)[0]
        stop.append(P + int(hit[0]) + 1 if hit.size else max_length)
    L_ref = min(max(stop), max_length, L_now)
    return ids[:, :L_ref]
