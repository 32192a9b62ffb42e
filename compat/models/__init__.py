"""Drop-in `models` package for the reference's scripts."""
