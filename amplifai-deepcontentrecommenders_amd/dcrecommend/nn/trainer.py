"""Trainer ABC of the reference (nn/trainer.py:6-32): fit / predict / score / save."""
from abc import ABC, abstractmethod


class Trainer(ABC):

    @abstractmethod
    def __init__(self):
        """Initialize the trainer."""

    @abstractmethod
    def fit(self):
        raise NotImplementedError("train is an abstract method.")

    @abstractmethod
    def predict(self):
        raise NotImplementedError("evaluate is an abstract method.")

    @abstractmethod
    def score(self):
        raise NotImplementedError("score is an abstract method.")

    @abstractmethod
    def save(self):
        raise NotImplementedError("save is an abstract method.")
