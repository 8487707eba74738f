"""The standalone ctypes stub in INTEGRATION.md §2 runs verbatim against libmdr_hip.so."""
import os
import re

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_stub_runs():
    import torch

    assert torch.cuda.is_available()
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        text = f.read()
    sec = text[text.index("## 2. The C ABI binding"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    code = code.replace('C.CDLL("marl-demandresponse_amd/mdr_amd/libmdr_hip.so")',
                        f'C.CDLL("{ROOT}/marl-demandresponse_amd/mdr_amd/libmdr_hip.so")')
    exec(compile(code, "INTEGRATION.md", "exec"), {})
