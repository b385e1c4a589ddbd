"""grayscott_amd.plot"""
