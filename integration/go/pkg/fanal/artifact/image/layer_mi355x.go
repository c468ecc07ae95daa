//go:build mi355x

// Image layers in the mi355x build: the secret analyzer takes a whole layer
// per GPU call instead of one file per Analyze.
//
// Artifact.inspectLayer (image.go:242-331) walks each uncompressed layer once
// and calls every analyzer per file.  For secrets that is one cgo call per
// file (analyzer/secret/secret_mi355x.go analyzes tar-header files per file).
// In the mi355x build NewArtifact tries newGPUSecrets; when the backend exists
// (a usable GPU and a ruleset the engine covers) the artifact's AnalyzerGroup
// is built with analyzer.TypeSecret disabled -- the per-file analyzer then
// never sees a layer file -- and inspectLayer makes two changes, marked below;
// without it nothing changes and Trivy's per-file analyzer runs as today:
//
//	layer, n, free, err := readLayer(rc)                          // (1) the layer, once, in C memory
//	defer free()
//	secrets, err := a.gpuSecrets.layerSecrets(layer, n, disabled) // (2) tsg_analyze_layer
//	... a.walker.Walk(bytes.NewReader(unsafe.Slice((*byte)(layer), n)), ...) // other analyzers as today
//	result.Secrets = append(result.Secrets, secrets...)           // before result.Sort()
//
// `disabled` is inspectLayer's own argument: the image's base layers carry
// analyzer.TypeSecret there (image.go:209-213) and yield no secrets, as the
// reference's AnalyzeFile skips the secret analyzer for them
// (analyzer.go:405-409).
//
// The walk inside the library applies the same skip rules and whiteout
// handling as walker.LayerTar (tar.go:35-117), and Required + Analyze of every
// regular file run in one tsg_analyze_layer call with the "/" path prefix of
// Dir "" (secret.go:95-98).  Executable mirror: trivy_amd/walker.py
// analyze_layer / analyze_layers (two engines per GPU take layers in turn;
// `disabled` marks base layers).
package image

/*
#include <stdlib.h>
*/
import "C"

import (
	"io"
	"os"
	"strconv"
	"unsafe"

	"golang.org/x/exp/slices"
	"golang.org/x/xerrors"

	"github.com/aquasecurity/trivy/pkg/fanal/analyzer"
	"github.com/aquasecurity/trivy/pkg/fanal/secret"
	"github.com/aquasecurity/trivy/pkg/fanal/types"
	"github.com/aquasecurity/trivy/pkg/fanal/walker"
)

// gpuSecrets is the secret analyzer of the mi355x build for image layers.
type gpuSecrets struct {
	backend    *secret.GPUBackend
	configPath string
	skipFiles  []string
	skipDirs   []string
}

// newGPUSecrets: nil when secret scanning is disabled for the artifact
// (nothing is created then) or the host has no usable backend (Trivy's
// per-file analyzer stays).
func newGPUSecrets(opt analyzer.AnalyzerOptions, wopt walker.Option) *gpuSecrets {
	if slices.Contains(opt.DisabledAnalyzers, analyzer.TypeSecret) {
		return nil
	}
	configPath := opt.SecretScannerOption.ConfigPath
	c, err := secret.ParseConfig(configPath)
	if err != nil {
		return nil // the per-file analyzer's Init reports the config error as today
	}
	device := 0
	if v, err := strconv.Atoi(os.Getenv("TRIVY_SECRET_GPU_DEVICE")); err == nil {
		device = v
	}
	be, err := secret.NewGPUBackend(secret.NewScanner(c), device)
	if err != nil {
		return nil
	}
	return &gpuSecrets{backend: be, configPath: configPath,
		skipFiles: walker.CleanSkipPaths(wopt.SkipFiles), skipDirs: walker.CleanSkipPaths(wopt.SkipDirs)}
}

// readLayer reads an uncompressed layer into C memory (outside the Go heap,
// so the library may read it during the call without a copy).
func readLayer(rc io.Reader) (unsafe.Pointer, int, func(), error) {
	size, capacity := 0, 64<<20
	buf := C.malloc(C.size_t(capacity))
	if buf == nil {
		return nil, 0, nil, xerrors.New("layer buffer: out of memory")
	}
	for {
		if size == capacity {
			capacity *= 2
			nb := C.realloc(buf, C.size_t(capacity))
			if nb == nil {
				C.free(buf)
				return nil, 0, nil, xerrors.New("layer buffer: out of memory")
			}
			buf = nb
		}
		n, err := rc.Read(unsafe.Slice((*byte)(buf), capacity)[size:])
		size += n
		if err == io.EOF {
			break
		}
		if err != nil {
			C.free(buf)
			return nil, 0, nil, xerrors.Errorf("layer read error: %w", err)
		}
	}
	return buf, size, func() { C.free(buf) }, nil
}

// layerSecrets: the layer's secrets (files with findings), as the per-file
// secret analyzer would have merged them into the layer's AnalysisResult;
// none for a layer whose `disabled` list holds TypeSecret (a base layer).
func (g *gpuSecrets) layerSecrets(layer unsafe.Pointer, n int, disabled []analyzer.Type) ([]types.Secret, error) {
	if slices.Contains(disabled, analyzer.TypeSecret) {
		return nil, nil
	}
	secrets, _, _, err := g.backend.AnalyzeLayer(layer, n, g.skipFiles, g.skipDirs, g.configPath)
	if err != nil {
		return nil, xerrors.Errorf("secret gpu layer analysis: %w", err)
	}
	return secrets, nil
}
