"""Drop-in for the reference's dataset package (dataset/kittiloader.py, dataset/nyuloader.py)."""
