"""User-level examples of the harp_amd programming model (ports of the reference's tutorials)."""
