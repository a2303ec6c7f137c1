"""Code <-> character serialisation, vectorised.

Same results as ``/root/reference/librispeech-mimi/utils.py:18-55`` (``codes_to_chars`` /
``chars_to_codes``; identical copies in the other ``*/utils.py``): codebook k's code c becomes the
character ``chr(unicode_offset + k*codebook_size + c)``, frames interleaved codebook-fastest
(``codes.T.reshape(-1)``).  The reference builds the string with a per-character ``chr`` loop
(``utils.py:36``), the host bottleneck at GPU encode rates; here the code points are formed in numpy and
the string is decoded from UTF-32 in one call.
"""
from __future__ import annotations

from typing import List, Optional, Union

import numpy as np
import torch

UNICODE_OFFSET: int = 0xE000
NUM_CODEBOOKS: int = 8
CODEBOOK_SIZE: int = 2048


def codes_to_codepoints(codes: Union[List[List[int]], np.ndarray, torch.Tensor], codebook_size: int,
                        copy_before_conversion: bool = True, unicode_offset: int = UNICODE_OFFSET) -> np.ndarray:
    """The code points ``codes_to_chars`` turns into characters, flat, in string order."""
    if isinstance(codes, list):
        codes = np.array(codes)
        copy_before_conversion = False
    elif isinstance(codes, torch.Tensor):
        codes = codes.cpu().numpy()
    if len(codes.shape) != 2:
        raise ValueError("codes must be a 2D array of shape (num_codebooks, seq_length).")
    if copy_before_conversion:
        codes = codes.copy()
    # the offset add stays in the codes' own dtype, row by row, exactly as the reference does it
    # (in place when copy_before_conversion=False; same overflow behaviour for narrow dtypes)
    for i in range(codes.shape[0]):
        codes[i] += unicode_offset + i * codebook_size
    return np.ascontiguousarray(codes.T.reshape(-1))


def codes_to_chars(codes: Union[List[List[int]], np.ndarray, torch.Tensor], codebook_size: int,
                   copy_before_conversion: bool = True, unicode_offset: int = UNICODE_OFFSET) -> str:
    flat = codes_to_codepoints(codes, codebook_size, copy_before_conversion, unicode_offset)
    if flat.size == 0:
        return ""
    if flat.dtype.kind not in "iu":
        return "".join([chr(c) for c in flat])  # chr() raises for floats exactly as the reference does
    lo, hi = int(flat.min()), int(flat.max())
    if lo < 0 or hi > 0x10FFFF or ((flat >= 0xD800) & (flat <= 0xDFFF)).any():
        return "".join([chr(c) for c in flat])  # out-of-range / surrogate code points: reference semantics
    return flat.astype("<u4").tobytes().decode("utf-32-le")


def chars_to_codes(chars: str, num_codebooks: int, codebook_size: int, return_tensors: Optional[str] = None,
                   unicode_offset: int = UNICODE_OFFSET):
    cp = np.frombuffer(chars.encode("utf-32-le"), dtype="<u4").astype(np.int64)
    codes = cp.reshape(-1, num_codebooks).T.copy()
    codes -= (unicode_offset + np.arange(num_codebooks, dtype=np.int64) * codebook_size)[:, None]
    if return_tensors is None:
        return codes.tolist()
    if return_tensors == "pt":
        return torch.tensor(codes)
    return codes


def audio_to_str(audio_numpy: np.ndarray, mimi_model, device: str) -> str:
    """``utils.audio_to_str`` (``librispeech-mimi/utils.py:58-69``) over the HIP model."""
    audio_tensor = torch.tensor(audio_numpy).to(device).unsqueeze(0)
    if len(audio_tensor.shape) == 2:
        audio_tensor = audio_tensor.unsqueeze(1)
    with torch.no_grad():
        audio_codes = mimi_model.encode(audio_tensor)
    codes = audio_codes[0][0].cpu()
    codes = codes[:NUM_CODEBOOKS, :]
    return codes_to_chars(codes, codebook_size=CODEBOOK_SIZE)
