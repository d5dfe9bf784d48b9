"""Evaluation harnesses (HellaSwag)."""
