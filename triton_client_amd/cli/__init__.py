"""Entry points (reference main.py, main3d.py, bag2d.py, bag3d.py, evaluate.py)."""
