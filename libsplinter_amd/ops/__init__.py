"""GPU operators (HIP/gfx950) exposed over torch tensors."""
