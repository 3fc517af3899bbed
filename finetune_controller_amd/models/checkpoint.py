"""Checkpoint I/O in the formats the controller's artifact contract expects.

The reference treats artifacts as opaque flat files synced from ``/data/artifacts`` by patterns
(``/root/reference/app/models/base/finetuning.py:94-97``: ``*.json *.yaml *.csv *.pt *.ckpt``) and
flattens sub-directories to basenames when zipping/presigning
(``/root/reference/app/utils/S3Handler.py:193,317``).  So everything here is written FLAT, with
unique names:

* LoRA / QLoRA: ``adapter_config.json`` (PEFT) + ``adapter_model.safetensors`` + ``adapter_model.pt``
  (same tensors; ``.pt`` is matched by the reference's default patterns, safetensors by ours);
* full fine-tune: ``config.json`` + ``model-0000i-of-0000n.safetensors`` shards +
  ``model.safetensors.index.json`` in Hugging Face naming (+ nothing pickled);
* resume: ``checkpoint_step{N}.pt`` (trainable tensors + optimizer flat state + data cursor),
  loaded with ``weights_only=True``.
"""
from __future__ import annotations

import glob
import json
import logging
import os
import re

import torch
from safetensors.torch import load_file, save_file

from .lora import LoRAConfig

_log = logging.getLogger("ftc.checkpoint")

PEFT_PREFIX = "base_model.model."

_LLAMA_SEG_MODULE = {"q_proj": "self_attn", "k_proj": "self_attn", "v_proj": "self_attn", "o_proj": "self_attn",
                     "gate_proj": "mlp", "up_proj": "mlp", "down_proj": "mlp"}
_GPT2_SEG_MODULE = {"q_proj": "attn.c_attn", "k_proj": "attn.c_attn", "v_proj": "attn.c_attn", "o_proj": "attn.c_proj",
                    "up_proj": "mlp.c_fc", "down_proj": "mlp.c_proj"}


def _layers(model):
    return model.layers if hasattr(model, "layers") else model.blocks


def adapter_state_dict(model) -> dict[str, torch.Tensor]:
    """PEFT-named LoRA tensors: ``...layers.{i}.self_attn.q_proj.lora_A.weight`` [r, in] / ``lora_B`` [out, r]."""
    sd = {}
    gpt2 = model.cfg.family == "gpt2"
    for i, layer in enumerate(_layers(model)):
        for pair in layer.lora.values():
            for seg, A_s, B_s in pair.segment_tensors():
                if gpt2:
                    base = f"{PEFT_PREFIX}transformer.h.{i}.{_GPT2_SEG_MODULE[seg]}.{seg}"
                else:
                    base = f"{PEFT_PREFIX}model.layers.{i}.{_LLAMA_SEG_MODULE[seg]}.{seg}"
                sd[f"{base}.lora_A.weight"] = A_s.detach().to(torch.bfloat16).contiguous().cpu()
                sd[f"{base}.lora_B.weight"] = B_s.detach().to(torch.bfloat16).contiguous().cpu()
    return sd


def _atomic(path: str, write):
    """``write(tmp)`` then rename onto ``path``: the s3-sync sidecar, which runs while the worker saves,
    never uploads a half-written weights file (its ``*.tmp`` exclude skips the temporary)."""
    tmp = path + ".tmp"
    write(tmp)
    os.replace(tmp, path)


def save_adapter(model, out_dir: str, base_model_name: str, lora: LoRAConfig, write_pt: bool = True) -> list[str]:
    os.makedirs(out_dir, exist_ok=True)
    sd = adapter_state_dict(model)
    files = []
    p = os.path.join(out_dir, "adapter_model.safetensors")
    _atomic(p, lambda t: save_file(sd, t, metadata={"format": "pt"}))
    files.append(p)
    if write_pt:
        p = os.path.join(out_dir, "adapter_model.pt")
        _atomic(p, lambda t: torch.save(sd, t))
        files.append(p)
    p = os.path.join(out_dir, "adapter_config.json")
    with open(p, "w") as f:
        json.dump(lora.to_peft(base_model_name), f, indent=2)
    files.append(p)
    return files


@torch.no_grad()
def load_adapter(model, path: str, layers_to_transform=None):
    """Load PEFT-named adapter tensors (safetensors or weights-only .pt) into the model's pairs.

    What the adapter must hold is derived from the ADAPTER, not from the model: its own segment names on
    the layers ``layers_to_transform`` names (argument, else ``adapter_config.json``'s, else the layers
    its keys cover).  A key with no LoRA slot in this model, or a lora_A without its lora_B, is refused; an
    expected (layer, segment) the file lacks (a truncated file) is refused; the model's slots the adapter
    does not train (other layers of a ``layers_to_transform`` adapter, other projections) get B = 0."""
    cfg_file = None
    if os.path.isdir(path):
        cfg_file = os.path.join(path, "adapter_config.json")
        st = os.path.join(path, "adapter_model.safetensors")
        path = st if os.path.exists(st) else os.path.join(path, "adapter_model.pt")
    else:
        cfg_file = os.path.join(os.path.dirname(path), "adapter_config.json")
    if layers_to_transform is None and cfg_file and os.path.exists(cfg_file):
        with open(cfg_file) as f:
            layers_to_transform = json.load(f).get("layers_to_transform")
    if isinstance(layers_to_transform, int):
        layers_to_transform = [layers_to_transform]
    sd = load_file(path) if path.endswith(".safetensors") else torch.load(path, map_location="cpu", weights_only=True)
    pat = re.compile(r"\.(?:layers|h)\.(\d+)\..*?\.(\w+_proj)\.lora_A\.weight$")
    layers = _layers(model)
    slots = {(i, seg) for i, layer in enumerate(layers) for pair in layer.lora.values() for seg in pair.names}
    done: set[tuple[int, str]] = set()
    for k, A in sd.items():
        m = pat.search(k)
        if not m:
            continue
        i, seg = int(m.group(1)), m.group(2)
        kb = k[: -len("lora_A.weight")] + "lora_B.weight"
        if (i, seg) not in slots:
            # an adapter of another model (more layers) or with targets this model was not built with:
            # refusing beats generating from a silently partial adapter
            raise ValueError(f"{os.path.basename(path)}: {k} has no LoRA slot in this model "
                             f"({len(layers)} layers; targets {sorted({s for _, s in slots})})")
        if kb not in sd:
            raise ValueError(f"{os.path.basename(path)}: {k} has no {kb.rsplit('.', 3)[-3]}.lora_B partner")
        for pair in layers[i].lora.values():
            if seg in pair.names:
                pair.load_segment(seg, A.to(pair.A.device, pair.A.dtype), sd[kb].to(pair.B.device, pair.B.dtype))
                done.add((i, seg))
    if not done:
        raise ValueError(f"{os.path.basename(path)}: no LoRA tensors found")
    segs = {seg for _, seg in done}
    on = set(layers_to_transform) if layers_to_transform is not None else {i for i, _ in done}
    expected = {(i, seg) for i in on for seg in segs}
    if expected - done:
        miss = sorted(expected - done)
        raise ValueError(f"{os.path.basename(path)}: {len(miss)} of {len(expected)} LoRA segments missing "
                         f"(e.g. layer {miss[0][0]} {miss[0][1]})")
    for i, seg in sorted(slots - done):  # slots this adapter does not train: no contribution
        for pair in layers[i].lora.values():
            if seg in pair.names:
                pair.zero_segment(seg)
    return len(done)


# ---------------- full model (HF naming) ----------------

def _llama_hf_tensors(model):
    cfg = model.cfg
    H, KV, D, Fd = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.ffn_dim
    yield "model.embed_tokens.weight", model.embed
    for i, l in enumerate(model.layers):
        p = f"model.layers.{i}."
        yield p + "input_layernorm.weight", l.attn_norm
        w = l.wqkv
        yield p + "self_attn.q_proj.weight", w[: H * D]
        yield p + "self_attn.k_proj.weight", w[H * D:(H + KV) * D]
        yield p + "self_attn.v_proj.weight", w[(H + KV) * D:]
        yield p + "self_attn.o_proj.weight", l.wo
        yield p + "post_attention_layernorm.weight", l.mlp_norm
        yield p + "mlp.gate_proj.weight", l.wgu[:Fd]
        yield p + "mlp.up_proj.weight", l.wgu[Fd:]
        yield p + "mlp.down_proj.weight", l.wdown
    yield "model.norm.weight", model.final_norm
    if not cfg.tie_embeddings:
        yield "lm_head.weight", model.lm_head


def _gpt2_hf_tensors(model):
    yield "transformer.wte.weight", model.wte
    yield "transformer.wpe.weight", model.wpe
    for i, b in enumerate(model.blocks):
        p = f"transformer.h.{i}."
        yield p + "ln_1.weight", b.ln1_w
        yield p + "ln_1.bias", b.ln1_b
        yield p + "attn.c_attn.weight", b.attn_w.t()  # HF Conv1D stores [in, out]
        yield p + "attn.c_attn.bias", b.attn_b
        yield p + "attn.c_proj.weight", b.proj_w.t()
        yield p + "attn.c_proj.bias", b.proj_b
        yield p + "ln_2.weight", b.ln2_w
        yield p + "ln_2.bias", b.ln2_b
        yield p + "mlp.c_fc.weight", b.fc_w.t()
        yield p + "mlp.c_fc.bias", b.fc_b
        yield p + "mlp.c_proj.weight", b.out_w.t()
        yield p + "mlp.c_proj.bias", b.out_b
    yield "transformer.ln_f.weight", model.lnf_w
    yield "transformer.ln_f.bias", model.lnf_b


def hf_tensors(model):
    return _gpt2_hf_tensors(model) if model.cfg.family == "gpt2" else _llama_hf_tensors(model)


def save_full(model, out_dir: str, shard_bytes: int = 5 * 1024**3, merge_lora: bool = True) -> list[str]:
    """HF-layout safetensors shards + index + config.json (LoRA merged in if present)."""
    os.makedirs(out_dir, exist_ok=True)
    from .lora import merge_pair_into

    merged = []
    if merge_lora and model.lora_cfg is not None and model.cfg.family != "gpt2":
        for l in model.layers:
            for name, pair in l.lora.items():
                if name in l.qweights:
                    continue
                merge_pair_into(l.base_weight(name).data, pair, +1.0)
                merged.append((l, name, pair))
    try:
        shards, cur, size = [], {}, 0
        for name, t in hf_tensors(model):
            t = t.detach().contiguous().cpu()
            nb = t.numel() * t.element_size()
            if cur and size + nb > shard_bytes:
                shards.append(cur)
                cur, size = {}, 0
            cur[name] = t
            size += nb
        if cur:
            shards.append(cur)
        files, weight_map = [], {}
        for i, sh in enumerate(shards):
            fn = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
            _atomic(os.path.join(out_dir, fn), lambda t, sh=sh: save_file(sh, t, metadata={"format": "pt"}))
            files.append(os.path.join(out_dir, fn))
            for k in sh:
                weight_map[k] = fn
        idx = os.path.join(out_dir, "model.safetensors.index.json")
        with open(idx, "w") as f:
            json.dump({"metadata": {}, "weight_map": weight_map}, f)
        cfgp = os.path.join(out_dir, "config.json")
        with open(cfgp, "w") as f:
            json.dump(model.cfg.to_hf_config(), f, indent=2)
        return files + [idx, cfgp]
    finally:
        for l, name, pair in merged:  # keep training state unmerged
            merge_pair_into(l.base_weight(name).data, pair, -1.0)
        if merged and hasattr(model, "invalidate_transposed"):
            model.invalidate_transposed()  # merge/unmerge round-trips W through bf16


@torch.no_grad()
def load_hf_checkpoint(model, path: str, strict: bool = True) -> int:
    """Load HF safetensors (sharded or single) into the packed layout; returns tensors loaded.

    Every target tensor must be filled exactly once with a matching shape: a missing tensor (wrong
    ``init_from``, a naming scheme this loader does not know, a partial shard set) or a shape
    mismatch raises instead of silently fine-tuning random-init weights.  Checkpoint tensors the
    model has no slot for (rotary ``inv_freq`` buffers, a tied ``lm_head``) are reported and skipped.
    ``strict=False`` only downgrades *missing* tensors to a warning."""
    files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
    files = [f for f in files if "adapter" not in os.path.basename(f)]
    if not files:
        raise FileNotFoundError(f"no *.safetensors weights under {path}")
    targets = dict(hf_tensors(model))
    loaded: set[str] = set()
    unexpected: list[str] = []
    for fp in files:
        sd = load_file(fp)
        for k, v in sd.items():
            if k not in targets and "transformer." + k in targets:
                k = "transformer." + k  # GPT-2 hub checkpoints saved from GPT2Model (no LM-head prefix)
            dst = targets.get(k)
            if dst is None:
                unexpected.append(k)
                continue
            if tuple(v.shape) != tuple(dst.shape):
                raise ValueError(f"{os.path.basename(fp)}: {k} has shape {tuple(v.shape)}, the model expects "
                                 f"{tuple(dst.shape)} (different architecture / config?)")
            if k in loaded:
                raise ValueError(f"{k} appears in more than one checkpoint shard")
            dst.copy_(v.to(dst.dtype))
            loaded.add(k)
    missing = sorted(set(targets) - loaded)
    if unexpected:
        _log.warning("load_hf_checkpoint: %d checkpoint tensors not used (e.g. %s)", len(unexpected),
                     ", ".join(unexpected[:3]))
    if missing:
        msg = (f"load_hf_checkpoint: {len(missing)} of {len(targets)} model tensors not found in {path} "
               f"(e.g. {', '.join(missing[:3])})")
        if strict:
            raise ValueError(msg)
        _log.warning(msg)
    if hasattr(model, "invalidate_transposed"):
        model.invalidate_transposed()
    return len(loaded)


# ---------------- resume checkpoints ----------------

def save_resume(path: str, step: int, opt, data_state: dict, extra: dict | None = None, opt_state: dict | None = None):
    opt_state = opt.state_dict() if opt_state is None else opt_state
    # trainable parameters in the compact per-parameter layout (no bucket padding): loadable at any
    # world size, with or without ZeRO-1
    st = {"step": step, "params": opt.export_params(),
          "opt": {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in opt_state.items()},
          "data": data_state, "extra": extra or {}}
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        torch.save(st, f)
        # on disk before the rename: the trainer deletes the previous resume point right after, so a
        # node crash must not leave the only checkpoint as a renamed file whose data never left the
        # page cache (the restarted pod would fail to read it on every attempt)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    fsync_dir(os.path.dirname(path) or ".")


def fsync_dir(d: str):
    """Make a rename in ``d`` durable (POSIX: the directory entry is only on disk after the directory's
    own fsync).  Best-effort where a filesystem refuses directory fsync."""
    try:
        fd = os.open(d, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def latest_resume(ckpt_dir: str) -> str | None:
    # only names this trainer writes (a stray checkpoint_step_best.pt must not break the restart)
    c = [p for p in glob.glob(os.path.join(ckpt_dir, "checkpoint_step*.pt"))
         if re.search(r"checkpoint_step(\d+)\.pt$", p)]
    if not c:
        return None
    return max(c, key=resume_step)


def resume_step(path: str) -> int:
    return int(re.search(r"checkpoint_step(\d+)\.pt$", path).group(1))


def read_resume(path: str) -> dict:
    st = torch.load(path, map_location="cpu", weights_only=True)
    if "params" not in st:
        raise ValueError(f"{os.path.basename(path)}: resume checkpoint predates the compact layout; "
                         "resume it with the build, world size and ZeRO setting that wrote it")
    return st


@torch.no_grad()
def load_resume(path: str, opt) -> dict:
    return apply_resume(read_resume(path), opt)


@torch.no_grad()
def apply_resume(st: dict, opt) -> dict:
    opt.import_params(st["params"])
    # compact state: the optimizer scatters it into its own layout (a sharded one keeps its part)
    opt.load_state_dict(st["opt"])
    return st
