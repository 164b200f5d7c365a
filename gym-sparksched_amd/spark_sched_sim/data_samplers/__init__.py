"""Dataset generation/packing and host-side reset sampling (tpch.py restated for the device layout)."""
