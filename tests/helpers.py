import torch


def _as_f64(t: torch.Tensor) -> torch.Tensor:
    t = t.detach().to("cpu")
    if t.is_complex():
        return torch.view_as_real(t.to(torch.complex128))
    return t.to(torch.float64)


def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    """Relative L2 error ||a - b|| / ||b|| (complex tensors compared as (re, im) pairs)."""
    a, b = _as_f64(a), _as_f64(b)
    if a.shape != b.shape and a.shape[:-1] == b.shape and a.shape[-1] == 2:
        b = torch.stack([b, torch.zeros_like(b)], -1)
    den = b.norm().item()
    num = (a - b).norm().item()
    return num / den if den > 0 else num
