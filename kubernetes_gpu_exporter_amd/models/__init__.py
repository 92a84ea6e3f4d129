"""Synthetic GPU pod workloads (GEMM pods, DP/TP/PP/SP/EP/CP/Ulysses trainer pods)."""
from .workloads import WORKLOADS, GemmPod, StepStats, TrainerPod, make, run

__all__ = ["WORKLOADS", "GemmPod", "StepStats", "TrainerPod", "make", "run"]
