import torch


def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    a = a.detach().to("cpu", torch.float64)
    b = b.detach().to("cpu", torch.float64)
    if a.is_complex() or b.is_complex():
        a = torch.view_as_real(a.to(torch.complex128)) if a.is_complex() else a
        b = torch.view_as_real(b.to(torch.complex128)) if b.is_complex() else b
    den = b.norm().item()
    num = (a - b).norm().item()
    return num / den if den > 0 else num
