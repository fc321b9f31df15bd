import torch


def perspective(vertices, angle=30.):
    """Perspective projection x/z/tan, y/z/tan (reference perspective.py:4-18).
    The reference converts degrees with pi ~= 3.1416; kept for parity."""
    assert vertices.ndim == 3
    if not torch.is_tensor(angle):
        angle = torch.as_tensor(angle, dtype=torch.float32, device=vertices.device)
    angle = (angle / 180. * 3.1416)[None].expand((vertices.shape[0],))
    width = torch.tan(angle)[:, None].expand(vertices.shape[:2])
    z = vertices[:, :, 2]
    x = vertices[:, :, 0] / z / width
    y = vertices[:, :, 1] / z / width
    return torch.stack((x, y, z), 2)
