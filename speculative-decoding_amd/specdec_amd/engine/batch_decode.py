"""engine/batch_decode.py:6-25: chat template + pad/truncate a prompt batch to [B, P]."""
from __future__ import annotations

from typing import List


def decode_batch_with_chat_template(tokenizer, prompts: List[str], max_length: int, chat: bool = True):
    if chat:
        prompts = [tokenizer.apply_chat_template([{"role": "user", "content": p}], add_generation_prompt=True,
                                                 tokenize=False) for p in prompts]
    enc = tokenizer(prompts, return_tensors="pt", padding=True, truncation=True, max_length=max_length)
    return enc.input_ids, enc.attention_mask
