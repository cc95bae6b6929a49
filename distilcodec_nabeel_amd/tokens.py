"""LLM token wire format of DistilCodec codes (host-only, no GPU).

Restates `DistilCodec.construct_audio_code` (distilcodec/distil_codec.py:200-265) and
`DistilCodec.audio_tokenize` (:532-543): code n of group g / residual r maps to
`{'content': '<|g{g}r{r}_{n+offset}|>', 'absolute_token_id': n + offset, 'in_codebook_id': n}`.
The offset advances by one codebook size per GROUP, not per (group, residual): in the reference the
`code_index_diff += codebook_size` sits after the residual loop (:219), so the residual codebooks of
one group share an id range (reproduced as is).  The table ends with 8 special audio tokens whose ids 5-7 carry the
reference's +7/+8/+9 absolute ids (kept verbatim, :253-262).
"""
from __future__ import annotations

_SPECIAL = [
    ("<|beginofaudio|>", "Audio output mode begin descriptor", 0),
    ("<|endofaudio|>", "Audio output mode end descriptor", 1),
    ("<|sil|>", "Audio silence descriptor", 2),
    ("<|inter_audio_begin|>", "Interleave Audio output mode begin descriptor", 3),
    ("<|inter_audio_end|>", "Interleave Audio output mode end descriptor", 4),
    ("<|cot_begin|>", "Cot begin descriptor", 7),
    ("<|cot_end|>", "Cot end descriptor", 8),
    ("<|unused600|>", "unused end descriptor", 9),
]


def construct_audio_code(n_groups: int, n_residual: int, codebook_size: int, tokens_id_offset: int = 0) -> dict:
    table = {}
    diff = tokens_id_offset
    for g in range(n_groups):
        for r in range(n_residual):
            codes = {str(n): {"content": f"<|g{g}r{r}_{n + diff}|>", "absolute_token_id": n + diff, "in_codebook_id": n}
                     for n in range(codebook_size)}
            table[f"g{g}r{r}"] = {"codebook_size": codebook_size, "audio_code_token": codes}
        diff += codebook_size  # once per group (distil_codec.py:219)
    table["special_audio_tokens"] = {
        str(diff + i): {"content": c, "description": d, "absolute_token_id": diff + a}
        for i, (c, d, a) in enumerate(_SPECIAL)
    }
    return table


def audio_tokenize(table: dict, codes: list, n_groups: int, n_residual: int) -> list:
    n_gr = n_groups * n_residual
    out = []
    for s in range(0, len(codes), n_gr):
        gr = codes[s: s + n_gr]
        for g, start in enumerate(range(0, len(gr), n_residual)):
            for r, code in enumerate(gr[start: start + n_residual]):
                out.append(table[f"g{g}r{r}"]["audio_code_token"][str(code)])
    return out
