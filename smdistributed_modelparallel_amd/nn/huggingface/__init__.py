"""HF transformers integration: predefined TP hooks and state-dict translators."""
