"""Drop-in replacement for the reference package workspace/src (MI355X HIP path)."""
