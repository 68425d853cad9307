'use strict';
// Return-shape contract of every feature (src/feature-info.js:1-65, with its export typo
// `module.exportts` fixed so the table is actually exported, and loudness/mfcc complete).
module.exports = {
  buffer: { type: 'array' },
  rms: { type: 'number' },
  energy: { type: 'number' },
  zcr: { type: 'number' },
  complexSpectrum: { type: 'multipleArrays', arrayNames: { 1: 'real', 2: 'imag' } },
  amplitudeSpectrum: { type: 'array' },
  powerSpectrum: { type: 'array' },
  spectralCentroid: { type: 'number' },
  spectralFlatness: { type: 'number' },
  spectralSlope: { type: 'number' },
  spectralRolloff: { type: 'number' },
  spectralSpread: { type: 'number' },
  spectralSkewness: { type: 'number' },
  spectralKurtosis: { type: 'number' },
  loudness: { type: 'multipleArrays', arrayNames: { 1: 'total', 2: 'specific' } },
  perceptualSpread: { type: 'number' },
  perceptualSharpness: { type: 'number' },
  mfcc: { type: 'array' },
};
