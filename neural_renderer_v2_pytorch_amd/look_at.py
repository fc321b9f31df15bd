import torch
import torch.nn.functional as F


def _as_batch(t, batch_size, device):
    if isinstance(t, (list, tuple)) or not torch.is_tensor(t):
        t = torch.as_tensor(t, dtype=torch.float32, device=device)
    if t.ndim == 1:
        t = t[None, :].expand((batch_size, t.shape[0]))
    return t


def look_at(vertices, viewpoints, at=None, up=None):
    """"Look at" view transform (reference look_at.py:5-44).

    Deliberate difference: the cross products take dim=-1 explicitly.  The reference calls
    torch.cross without `dim`, which at batch size 3 crosses along the batch axis and returns a
    wrong rotation (SURVEY.md section 8a hazards); every other batch size is unchanged."""
    assert vertices.ndim == 3
    device = vertices.device
    B = vertices.shape[0]
    at = _as_batch([0, 0, 0] if at is None else at, B, device)
    up = _as_batch([0, 1, 0] if up is None else up, B, device)
    viewpoints = _as_batch(viewpoints, B, device)

    z_axis = F.normalize(at - viewpoints)
    x_axis = F.normalize(torch.cross(up, z_axis, dim=-1))
    y_axis = F.normalize(torch.cross(z_axis, x_axis, dim=-1))
    r = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), 1)
    if r.shape[0] != B:
        r = r.expand((B, 3, 3))
    if vertices.shape != viewpoints.shape:
        viewpoints = viewpoints[:, None, :].expand(vertices.shape)
    return torch.matmul(vertices - viewpoints, r.permute(0, 2, 1))
