"""Reference application drivers restated on spartan_amd.expr (spartan/examples)."""
