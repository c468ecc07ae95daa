//go:build mi355x

// The image-config secret analyzer of the mi355x build
// (imgconf/secret/secret.go:26-62): the same rendering of the image's
// v1.ConfigFile (json.MarshalIndent(cfg, "  ", "")) scanned as one file named
// "config.json", on the GPU engine of this process.  The engine is created
// at the first Analyze (the constructor runs for every image, secret
// scanning or not) and shared by every image of the process; a host without a
// usable backend keeps the pure-Go Scanner the reference uses.
// Executable mirror: trivy_amd/imgconf.py ImageConfigSecretAnalyzer
// (tests/test_imgconf.py).
package secret

import (
	"context"
	"encoding/json"
	"os"
	"strconv"
	"sync"

	"golang.org/x/xerrors"

	"github.com/aquasecurity/trivy/pkg/fanal/analyzer"
	"github.com/aquasecurity/trivy/pkg/fanal/secret"
	"github.com/aquasecurity/trivy/pkg/log"
)

func init() {
	analyzer.RegisterConfigAnalyzer(analyzer.TypeImageConfigSecret, newGPUConfigAnalyzer)
}

// one backend per config path per process
var (
	backendsMu sync.Mutex
	backends   = map[string]*secret.GPUBackend{}
	noBackend  = map[string]bool{}
)

type gpuConfigAnalyzer struct {
	secretAnalyzer // scanner: the pure-Go Scanner (fallback)
	configPath     string
}

func newGPUConfigAnalyzer(opts analyzer.ConfigAnalyzerOptions) (analyzer.ConfigAnalyzer, error) {
	a, err := newSecretAnalyzer(opts) // ParseConfig + NewScanner (secret.go:26-38)
	if err != nil {
		return nil, err
	}
	return &gpuConfigAnalyzer{secretAnalyzer: *a.(*secretAnalyzer), configPath: opts.SecretScannerOption.ConfigPath}, nil
}

func (a *gpuConfigAnalyzer) backend() *secret.GPUBackend {
	backendsMu.Lock()
	defer backendsMu.Unlock()
	if be, ok := backends[a.configPath]; ok {
		return be
	}
	if noBackend[a.configPath] {
		return nil
	}
	device := 0
	if v, err := strconv.Atoi(os.Getenv("TRIVY_SECRET_GPU_DEVICE")); err == nil {
		device = v
	}
	be, err := secret.NewGPUBackend(a.scanner, device)
	if err != nil {
		log.Info("MI355X secret backend unavailable for image configs", log.Err(err))
		noBackend[a.configPath] = true
		return nil
	}
	backends[a.configPath] = be
	return be
}

func (a *gpuConfigAnalyzer) Analyze(ctx context.Context, input analyzer.ConfigAnalysisInput) (*analyzer.ConfigAnalysisResult, error) {
	if input.Config == nil {
		return nil, nil
	}
	be := a.backend()
	if be == nil {
		return a.secretAnalyzer.Analyze(ctx, input)
	}
	b, err := json.MarshalIndent(input.Config, "  ", "")
	if err != nil {
		return nil, xerrors.Errorf("json marshal error: %w", err)
	}
	out, err := be.ScanBatch([]secret.ScanArgs{{FilePath: "config.json", Content: b}})
	if err != nil {
		return a.secretAnalyzer.Analyze(ctx, input) // this image: the pure-Go Scanner
	}
	result := out[0]
	if len(result.Findings) == 0 {
		log.Debug("No secrets found in container image config")
		return nil, nil
	}
	return &analyzer.ConfigAnalysisResult{Secret: &result}, nil
}
