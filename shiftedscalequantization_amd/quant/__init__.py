"""Python mirror of the reference quant/ package (filled in below)."""
