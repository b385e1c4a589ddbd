"""grayscott_amd.analysis"""
