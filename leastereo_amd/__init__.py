"""MI355X-native LEAStereo inference hot path."""
