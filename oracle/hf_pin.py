"""Independent implementation used to pin ``clip_ref`` — TEST INFRASTRUCTURE.

Loads the oracle's seeded open_clip-named weights into HF ``transformers``
``CLIPVisionModelWithProjection`` / ``CLIPTextModelWithProjection`` (same
architecture as open_clip's OpenAI-style ViT / text transformer), so the two
implementations can be compared on identical parameters.  Imported only by
``tests/`` and ``tests/golden/make_golden.py``.
"""
from __future__ import annotations

import numpy as np


def _split_block(P, src, dst, D, sd):
    w = P[src + "attn.in_proj_weight"]
    b = P[src + "attn.in_proj_bias"]
    for j, nm in enumerate(("q_proj", "k_proj", "v_proj")):
        sd[dst + f"self_attn.{nm}.weight"] = w[j * D:(j + 1) * D]
        sd[dst + f"self_attn.{nm}.bias"] = b[j * D:(j + 1) * D]
    sd[dst + "self_attn.out_proj.weight"] = P[src + "attn.out_proj.weight"]
    sd[dst + "self_attn.out_proj.bias"] = P[src + "attn.out_proj.bias"]
    sd[dst + "layer_norm1.weight"] = P[src + "ln_1.weight"]
    sd[dst + "layer_norm1.bias"] = P[src + "ln_1.bias"]
    sd[dst + "layer_norm2.weight"] = P[src + "ln_2.weight"]
    sd[dst + "layer_norm2.bias"] = P[src + "ln_2.bias"]
    sd[dst + "mlp.fc1.weight"] = P[src + "mlp.c_fc.weight"]
    sd[dst + "mlp.fc1.bias"] = P[src + "mlp.c_fc.bias"]
    sd[dst + "mlp.fc2.weight"] = P[src + "mlp.c_proj.weight"]
    sd[dst + "mlp.fc2.bias"] = P[src + "mlp.c_proj.bias"]


def hf_vision(P, v, dtype="float64"):
    import torch
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection
    cfg = CLIPVisionConfig(hidden_size=v.width, intermediate_size=v.mlp_width,
                           num_hidden_layers=v.layers, num_attention_heads=v.heads,
                           image_size=v.image_size, patch_size=v.patch_size,
                           projection_dim=v.embed_dim, hidden_act=v.act,
                           layer_norm_eps=v.ln_eps, attn_implementation="eager")
    m = CLIPVisionModelWithProjection(cfg).eval()
    sd = {
        "vision_model.embeddings.patch_embedding.weight": P["visual.conv1.weight"],
        "vision_model.embeddings.class_embedding": P["visual.class_embedding"],
        "vision_model.embeddings.position_embedding.weight": P["visual.positional_embedding"],
        "vision_model.pre_layrnorm.weight": P["visual.ln_pre.weight"],
        "vision_model.pre_layrnorm.bias": P["visual.ln_pre.bias"],
        "vision_model.post_layernorm.weight": P["visual.ln_post.weight"],
        "vision_model.post_layernorm.bias": P["visual.ln_post.bias"],
        "visual_projection.weight": P["visual.proj"].T,
    }
    for i in range(v.layers):
        _split_block(P, f"visual.transformer.resblocks.{i}.",
                     f"vision_model.encoder.layers.{i}.", v.width, sd)
    sd = {k: torch.from_numpy(np.ascontiguousarray(a)) for k, a in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    assert not missing and not unexpected, (missing, unexpected)
    return m.to(getattr(torch, dtype))


def hf_text(P, t, dtype="float64"):
    import torch
    from transformers import CLIPTextConfig, CLIPTextModelWithProjection
    cfg = CLIPTextConfig(vocab_size=t.vocab_size, hidden_size=t.width,
                         intermediate_size=t.mlp_width, num_hidden_layers=t.layers,
                         num_attention_heads=t.heads, max_position_embeddings=t.context_length,
                         projection_dim=t.embed_dim, hidden_act=t.act, layer_norm_eps=t.ln_eps,
                         eos_token_id=2,  # legacy switch: pool at argmax(input_ids)
                         attn_implementation="eager")
    m = CLIPTextModelWithProjection(cfg).eval()
    sd = {
        "text_model.embeddings.token_embedding.weight": P["token_embedding.weight"],
        "text_model.embeddings.position_embedding.weight": P["positional_embedding"],
        "text_model.final_layer_norm.weight": P["ln_final.weight"],
        "text_model.final_layer_norm.bias": P["ln_final.bias"],
        "text_projection.weight": P["text_projection"].T,
    }
    for i in range(t.layers):
        _split_block(P, f"transformer.resblocks.{i}.", f"text_model.encoder.layers.{i}.", t.width, sd)
    sd = {k: torch.from_numpy(np.ascontiguousarray(a)) for k, a in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    assert not missing and not unexpected, (missing, unexpected)
    return m.to(getattr(torch, dtype))


def hf_siglip_text(P, t, dtype="float64"):
    """HF SiglipTextModel (no causal mask, last-position pooling, `head` Linear) with the
    open_clip-named seeded weights of a SigLIP2-form text tower (text_cfg no_causal_mask,
    pool_type "last", proj_bias; transformers' Siglip2 text tower is the same module)."""
    import torch
    from transformers import SiglipTextConfig, SiglipTextModel
    assert not t.causal and t.pool == "last" and t.proj_bias
    cfg = SiglipTextConfig(vocab_size=t.vocab_size, hidden_size=t.width, intermediate_size=t.mlp_width,
                           num_hidden_layers=t.layers, num_attention_heads=t.heads,
                           max_position_embeddings=t.context_length, hidden_act="gelu_pytorch_tanh",
                           layer_norm_eps=t.ln_eps, projection_size=t.embed_dim, bos_token_id=None,
                           eos_token_id=None, pad_token_id=None, attn_implementation="eager")
    m = SiglipTextModel(cfg).eval()
    sd = {
        "text_model.embeddings.token_embedding.weight": P["token_embedding.weight"],
        "text_model.embeddings.position_embedding.weight": P["positional_embedding"],
        "text_model.final_layer_norm.weight": P["ln_final.weight"],
        "text_model.final_layer_norm.bias": P["ln_final.bias"],
        "text_model.head.weight": P["text_projection.weight"],
        "text_model.head.bias": P["text_projection.bias"],
    }
    for i in range(t.layers):
        _split_block(P, f"transformer.resblocks.{i}.", f"text_model.encoder.layers.{i}.", t.width, sd)
    pre = "" if any(k.startswith("embeddings.") for k in m.state_dict()) else "text_model."
    sd = {pre + k[len("text_model."):]: torch.from_numpy(np.ascontiguousarray(x)) for k, x in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    assert not missing and not unexpected, (missing, unexpected)
    return m.to(getattr(torch, dtype))


def hf_siglip_encode_text(m, ids):
    import torch
    with torch.no_grad():
        e = m(input_ids=torch.from_numpy(np.asarray(ids, np.int64))).pooler_output
        e = torch.nn.functional.normalize(e, dim=-1)
    return e.double().numpy()


def hf_encode_image(m, pixels):
    import torch
    dt = next(m.parameters()).dtype
    with torch.no_grad():
        e = m(pixel_values=torch.from_numpy(np.asarray(pixels)).to(dt)).image_embeds
        e = torch.nn.functional.normalize(e, dim=-1)
    return e.double().numpy()


def hf_encode_text(m, ids):
    import torch
    with torch.no_grad():
        e = m(input_ids=torch.from_numpy(np.asarray(ids, np.int64))).text_embeds
        e = torch.nn.functional.normalize(e, dim=-1)
    return e.double().numpy()


def hf_siglip_vision(P, v, dtype="float64"):
    """HF SiglipVisionModel (vision_use_head: MAP head) with the timm-named seeded weights:
    qkv splits into q/k/v_proj; the attention-pool latent is the HF probe and [q | kv] its
    packed nn.MultiheadAttention in_proj."""
    import torch
    from transformers import SiglipVisionConfig, SiglipVisionModel
    cfg = SiglipVisionConfig(hidden_size=v.width, intermediate_size=v.mlp_width, num_hidden_layers=v.layers,
                             num_attention_heads=v.heads, image_size=v.image_size, patch_size=v.patch_size,
                             hidden_act="gelu_pytorch_tanh", layer_norm_eps=v.ln_eps, attn_implementation="eager")
    m = SiglipVisionModel(cfg).eval()
    t, a, D = "visual.trunk.", "visual.trunk.attn_pool.", v.width
    sd = {
        "vision_model.embeddings.patch_embedding.weight": P[t + "patch_embed.proj.weight"],
        "vision_model.embeddings.patch_embedding.bias": P[t + "patch_embed.proj.bias"],
        "vision_model.embeddings.position_embedding.weight": P[t + "pos_embed"][0],
        "vision_model.post_layernorm.weight": P[t + "norm.weight"],
        "vision_model.post_layernorm.bias": P[t + "norm.bias"],
        "vision_model.head.probe": P[a + "latent"],
        "vision_model.head.attention.in_proj_weight": np.concatenate([P[a + "q.weight"], P[a + "kv.weight"]]),
        "vision_model.head.attention.in_proj_bias": np.concatenate([P[a + "q.bias"], P[a + "kv.bias"]]),
        "vision_model.head.attention.out_proj.weight": P[a + "proj.weight"],
        "vision_model.head.attention.out_proj.bias": P[a + "proj.bias"],
        "vision_model.head.layernorm.weight": P[a + "norm.weight"],
        "vision_model.head.layernorm.bias": P[a + "norm.bias"],
        "vision_model.head.mlp.fc1.weight": P[a + "mlp.fc1.weight"],
        "vision_model.head.mlp.fc1.bias": P[a + "mlp.fc1.bias"],
        "vision_model.head.mlp.fc2.weight": P[a + "mlp.fc2.weight"],
        "vision_model.head.mlp.fc2.bias": P[a + "mlp.fc2.bias"],
    }
    for i in range(v.layers):
        src, dst = f"{t}blocks.{i}.", f"vision_model.encoder.layers.{i}."
        w, b = P[src + "attn.qkv.weight"], P[src + "attn.qkv.bias"]
        for j, nm in enumerate(("q_proj", "k_proj", "v_proj")):
            sd[dst + f"self_attn.{nm}.weight"] = w[j * D:(j + 1) * D]
            sd[dst + f"self_attn.{nm}.bias"] = b[j * D:(j + 1) * D]
        for hf, tm in (("self_attn.out_proj", "attn.proj"), ("layer_norm1", "norm1"), ("layer_norm2", "norm2"),
                       ("mlp.fc1", "mlp.fc1"), ("mlp.fc2", "mlp.fc2")):
            sd[dst + hf + ".weight"] = P[src + tm + ".weight"]
            sd[dst + hf + ".bias"] = P[src + tm + ".bias"]
    pre = "" if any(k.startswith("embeddings.") for k in m.state_dict()) else "vision_model."
    sd = {pre + k[len("vision_model."):]: torch.from_numpy(np.ascontiguousarray(x)) for k, x in sd.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    assert not missing and not unexpected, (missing, unexpected)
    return m.to(getattr(torch, dtype))


def hf_siglip_encode_image(m, pixels):
    import torch
    dt = next(m.parameters()).dtype
    with torch.no_grad():
        e = m(pixel_values=torch.from_numpy(np.asarray(pixels)).to(dt)).pooler_output
        e = torch.nn.functional.normalize(e, dim=-1)
    return e.double().numpy()
